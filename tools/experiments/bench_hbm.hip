// HBM ceiling for the scrypt ROMix access pattern on gfx950 (no compute):
//   read : random full 128-B lines inside a per-wave 8 MiB region (8 lanes x 16 B per line),
//          `inflight` independent lines per octet per step (the ROMix lookup has 1 per hash)
//   write: sequential full lines per wave region (the ROMix write phase)
//   mixed: 1 random line read + 1 sequential line write per octet per step (ROMix gap-1 ratio)
// Prints achieved TB/s per pattern so the 16.1 MH/s x 256 KiB = 4.2 TB/s of the cooperative
// ROMix can be priced against what the memory system gives this pattern.
// Build: hipcc --offload-arch=gfx950 -O3 tools/bench_hbm.hip -o build/bench_hbm
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

constexpr uint64_t kRegion = 8ull << 20;  // bytes per wave (ROMix gap-1 pad)
typedef unsigned nv4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xs(uint32_t x) {
  x ^= x << 13;
  x ^= x >> 17;
  x ^= x << 5;
  return x;
}

template <int INFLIGHT>
__global__ __launch_bounds__(256) void rand_read(const uint4* __restrict__ V, uint32_t* out, int steps) {
  const uint64_t gl = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t wave = gl >> 6;
  const uint32_t lane = gl & 63, octet = lane >> 3, slot = lane & 7;
  const char* base = reinterpret_cast<const char*>(V) + wave * kRegion;
  uint32_t s = uint32_t(wave * 8 + octet) * 2654435761u + 12345u;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int i = 0; i < steps; ++i) {
    uint4 v[INFLIGHT];
#pragma unroll
    for (int k = 0; k < INFLIGHT; ++k) {
      s = xs(s);
      const uint32_t line = s & (uint32_t(kRegion / 128) - 1);
      v[k] = *reinterpret_cast<const uint4*>(base + uint64_t(line) * 128 + slot * 16);
    }
#pragma unroll
    for (int k = 0; k < INFLIGHT; ++k) { acc.x ^= v[k].x; acc.y ^= v[k].y; acc.z ^= v[k].z; acc.w ^= v[k].w; }
  }
  out[gl] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <bool NT>
__global__ __launch_bounds__(256) void seq_write(uint4* __restrict__ V, int steps) {
  const uint64_t gl = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t wave = gl >> 6;
  const uint32_t lane = gl & 63;
  char* base = reinterpret_cast<char*>(V) + wave * kRegion;
  for (int i = 0; i < steps; ++i) {
    // 8 instructions per step, each writing 8 full lines (1 KiB contiguous per instruction)
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const uint64_t off = (uint64_t(i) * 8192 + r * 1024 + lane * 16) % kRegion;
      uint4* p = reinterpret_cast<uint4*>(base + off);
      const uint4 v = make_uint4(i, r, lane, 7);
      if constexpr (NT) __builtin_nontemporal_store(nv4{v.x, v.y, v.z, v.w}, reinterpret_cast<nv4*>(p)); else *p = v;
    }
  }
}

template <bool NT>
__global__ __launch_bounds__(256) void mixed(uint4* __restrict__ V, uint32_t* out, int steps) {
  const uint64_t gl = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t wave = gl >> 6;
  const uint32_t lane = gl & 63, octet = lane >> 3, slot = lane & 7;
  char* base = reinterpret_cast<char*>(V) + wave * kRegion;
  uint32_t s = uint32_t(wave * 8 + octet) * 2654435761u + 777u;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (int i = 0; i < steps; ++i) {
    // write: this step's 8 KiB (one line per octet per instruction, 8 instructions)
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const uint64_t off = (uint64_t(i) * 8192 + r * 1024 + lane * 16) % kRegion;
      uint4* p = reinterpret_cast<uint4*>(base + off);
      const uint4 w = make_uint4(i, r, lane, acc.x);
      if constexpr (NT) __builtin_nontemporal_store(nv4{w.x, w.y, w.z, w.w}, reinterpret_cast<nv4*>(p)); else *p = w;
    }
    // read: 8 random lines per octet (= one 128-B lookup per owner lane, 64 per wave)
    uint4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s = xs(s);
      const uint32_t line = s & (uint32_t(kRegion / 128) - 1);
      v[k] = *reinterpret_cast<const uint4*>(base + uint64_t(line) * 128 + slot * 16);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) { acc.x ^= v[k].x; acc.y ^= v[k].y; acc.z ^= v[k].z; acc.w ^= v[k].w; }
  }
  out[gl] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

static void ck(hipError_t e, const char* w) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "%s: %s\n", w, hipGetErrorString(e));
    std::exit(1);
  }
}

int main(int argc, char** argv) {
  const int grid = argc > 1 ? std::atoi(argv[1]) : 2048;
  const int steps = argc > 2 ? std::atoi(argv[2]) : 256;
  const uint64_t waves = uint64_t(grid) * 4;
  const uint64_t bytes = waves * kRegion;
  uint4* V = nullptr;
  uint32_t* out = nullptr;
  ck(hipMalloc(&V, bytes), "malloc pad");
  ck(hipMalloc(&out, uint64_t(grid) * 256 * 4), "malloc out");
  ck(hipMemset(V, 1, bytes), "memset");
  hipEvent_t a, b;
  ck(hipEventCreate(&a), "ev");
  ck(hipEventCreate(&b), "ev");
  auto timeit = [&](const char* name, auto launch, double bytes_moved) {
    for (int rep = 0; rep < 3; ++rep) {
      ck(hipEventRecord(a, nullptr), "rec");
      launch();
      ck(hipGetLastError(), "launch");
      ck(hipEventRecord(b, nullptr), "rec");
      ck(hipEventSynchronize(b), "sync");
      float ms = 0;
      ck(hipEventElapsedTime(&ms, a, b), "elapsed");
      std::printf("{\"pattern\": \"%s\", \"grid\": %d, \"steps\": %d, \"ms\": %.3f, \"TBps\": %.3f}\n", name, grid,
                  steps, ms, bytes_moved / (ms * 1e-3) / 1e12);
    }
  };
  const double lanes = double(grid) * 256;
  timeit("rand_read_1", [&] { hipLaunchKernelGGL(rand_read<1>, dim3(grid), dim3(256), 0, nullptr, V, out, steps * 8); },
         lanes * steps * 8 * 16);
  timeit("rand_read_4", [&] { hipLaunchKernelGGL(rand_read<4>, dim3(grid), dim3(256), 0, nullptr, V, out, steps * 2); },
         lanes * steps * 8 * 16);
  timeit("seq_write", [&] { hipLaunchKernelGGL(seq_write<false>, dim3(grid), dim3(256), 0, nullptr, V, steps); },
         lanes * steps * 8 * 16);
  timeit("seq_write_nt", [&] { hipLaunchKernelGGL(seq_write<true>, dim3(grid), dim3(256), 0, nullptr, V, steps); },
         lanes * steps * 8 * 16);
  timeit("mixed_1r1w", [&] { hipLaunchKernelGGL(mixed<false>, dim3(grid), dim3(256), 0, nullptr, V, out, steps); },
         lanes * steps * 16 * 16);
  timeit("mixed_1r1w_nt", [&] { hipLaunchKernelGGL(mixed<true>, dim3(grid), dim3(256), 0, nullptr, V, out, steps); },
         lanes * steps * 16 * 16);
  ck(hipFree(V), "free");
  ck(hipFree(out), "free");
  return 0;
}
