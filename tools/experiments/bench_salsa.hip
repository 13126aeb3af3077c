// Microbenchmark: BlockMix_salsa20/8 issue rate on gfx950 with no memory traffic.
// Separates "ROMix is latency/memory bound" from "the Salsa instruction stream itself
// issues slower than one VALU per 4 cycles". Variants:
//   1: one hash per lane (the production ROMix arithmetic)
//   2: two independent hashes per lane, salsa rounds interleaved (2x ILP, 2x VGPR)
// Build: hipcc --offload-arch=gfx950 -O3 -I../csrc/kernels tools/bench_salsa.hip -o build/bench_salsa
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "cdna_bitops.h"

using otedama_dev::rol;

#define QR(a, b, c, d)                                                                        \
  b ^= rol(a + d, 7);                                                                         \
  c ^= rol(b + a, 9);                                                                         \
  d ^= rol(c + b, 13);                                                                        \
  a ^= rol(d + c, 18);

__device__ __forceinline__ void salsa(uint32_t* B) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = B[i];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    QR(x[0], x[4], x[8], x[12]) QR(x[5], x[9], x[13], x[1]) QR(x[10], x[14], x[2], x[6]) QR(x[15], x[3], x[7], x[11])
    QR(x[0], x[1], x[2], x[3]) QR(x[5], x[6], x[7], x[4]) QR(x[10], x[11], x[8], x[9]) QR(x[15], x[12], x[13], x[14])
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) B[i] += x[i];
}

__device__ __forceinline__ void salsa2(uint32_t* B, uint32_t* C) {
  uint32_t x[16], y[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { x[i] = B[i]; y[i] = C[i]; }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    QR(x[0], x[4], x[8], x[12]) QR(y[0], y[4], y[8], y[12]) QR(x[5], x[9], x[13], x[1]) QR(y[5], y[9], y[13], y[1])
    QR(x[10], x[14], x[2], x[6]) QR(y[10], y[14], y[2], y[6]) QR(x[15], x[3], x[7], x[11]) QR(y[15], y[3], y[7], y[11])
    QR(x[0], x[1], x[2], x[3]) QR(y[0], y[1], y[2], y[3]) QR(x[5], x[6], x[7], x[4]) QR(y[5], y[6], y[7], y[4])
    QR(x[10], x[11], x[8], x[9]) QR(y[10], y[11], y[8], y[9]) QR(x[15], x[12], x[13], x[14]) QR(y[15], y[12], y[13], y[14])
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) { B[i] += x[i]; C[i] += y[i]; }
}

__device__ __forceinline__ void blockmix(uint32_t* X) {
#pragma unroll
  for (int k = 0; k < 16; ++k) X[k] ^= X[16 + k];
  salsa(X);
#pragma unroll
  for (int k = 0; k < 16; ++k) X[16 + k] ^= X[k];
  salsa(X + 16);
}

__device__ __forceinline__ void blockmix2(uint32_t* X, uint32_t* Y) {
#pragma unroll
  for (int k = 0; k < 16; ++k) { X[k] ^= X[16 + k]; Y[k] ^= Y[16 + k]; }
  salsa2(X, Y);
#pragma unroll
  for (int k = 0; k < 16; ++k) { X[16 + k] ^= X[k]; Y[16 + k] ^= Y[k]; }
  salsa2(X + 16, Y + 16);
}

__global__ __launch_bounds__(256) void bm1(uint32_t* out, int iters) {
  uint32_t X[32];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 32; ++i) X[i] = t * 0x9E3779B9u + uint32_t(i);
  for (int it = 0; it < iters; ++it) blockmix(X);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) acc ^= X[i];
  out[t] = acc;
}

__global__ __launch_bounds__(256) void bm2(uint32_t* out, int iters) {
  uint32_t X[32], Y[32];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 32; ++i) { X[i] = t * 0x9E3779B9u + uint32_t(i); Y[i] = X[i] ^ 0x5bd1e995u; }
  for (int it = 0; it < iters; ++it) blockmix2(X, Y);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) acc ^= X[i] ^ Y[i];
  out[t] = acc;
}

static void check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
    std::exit(1);
  }
}

int main(int argc, char** argv) {
  const int grid = argc > 1 ? std::atoi(argv[1]) : 2048;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 2048;
  uint32_t* out = nullptr;
  check(hipMalloc(&out, size_t(grid) * 256 * 4), "malloc");
  hipEvent_t a, b;
  check(hipEventCreate(&a), "ev");
  check(hipEventCreate(&b), "ev");
  for (int variant = 1; variant <= 2; ++variant) {
    for (int rep = 0; rep < 3; ++rep) {
      check(hipEventRecord(a, nullptr), "rec");
      if (variant == 1)
        hipLaunchKernelGGL(bm1, dim3(grid), dim3(256), 0, nullptr, out, iters);
      else
        hipLaunchKernelGGL(bm2, dim3(grid), dim3(256), 0, nullptr, out, iters);
      check(hipGetLastError(), "launch");
      check(hipEventRecord(b, nullptr), "rec");
      check(hipEventSynchronize(b), "sync");
      float ms = 0;
      check(hipEventElapsedTime(&ms, a, b), "elapsed");
      const double blockmixes = double(grid) * 256 * iters * variant;
      // 2048 BlockMix = one scrypt(1024,1,1) hash at lookup gap 1
      std::printf("{\"variant\": %d, \"grid\": %d, \"iters\": %d, \"ms\": %.3f, \"blockmix_per_s\": %.4g, "
                  "\"hash_equiv_mhs\": %.3f}\n",
                  variant, grid, iters, ms, blockmixes / (ms * 1e-3), blockmixes / 2048.0 / (ms * 1e-3) / 1e6);
    }
  }
  check(hipFree(out), "free");
  return 0;
}
