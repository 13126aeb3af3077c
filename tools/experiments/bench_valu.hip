// VALU issue-rate microbenchmark for gfx950: cycles per wave64 instruction per SIMD, by op and occupancy.
//
// Why: every hash kernel here is VALU-issue bound, and the per-op cost decides which form of a round is
// cheapest (VOP2 pairs vs VOP3 fused ops, operand VGPR banks, SGPR operands). Each wave runs `iters`
// bodies of kBodyLen (64) independent instructions of one op (tools/bench_valu_bodies.h) on fixed registers; B blocks
// of 256 threads per CU put B waves on every SIMD. Reported per (op, B):
//   cyc  = s_memtime cycles of a block / (B * instructions per wave)  -> SIMD cycles per wave-instruction
//   wall = same from hipEvent time at the device's max clock
// Build: hipcc --offload-arch=gfx950 -O3 tools/bench_valu.hip -o build/bench_valu
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "bench_valu_bodies.h"

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

#define CLOBBERS                                                                                               \
  "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", \
      "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "s8", "s10", "s11", "vcc"

template <int OP>
__device__ __forceinline__ void body() {
#define CASE(n) \
  if constexpr (OP == n) asm volatile(BODY_##n ::: CLOBBERS);
  FOR_EACH_OP(CASE)
#undef CASE
}

template <int OP>
__global__ __launch_bounds__(256) void k_valu(unsigned long long* cyc, uint32_t* out, int iters) {
  const uint32_t seed = threadIdx.x * 2654435761u ^ blockIdx.x;
  asm volatile(
      "v_mov_b32 v40, %0\n\tv_add_u32 v41, 1, %0\n\tv_add_u32 v42, 2, %0\n\tv_add_u32 v43, 3, %0\n\t"
      "v_add_u32 v44, 4, %0\n\tv_add_u32 v45, 5, %0\n\tv_add_u32 v46, 6, %0\n\tv_add_u32 v47, 7, %0\n\t"
      "v_add_u32 v48, 8, %0\n\tv_mov_b32 v20, %0\n\ts_mov_b32 s8, 0x9e3779b9" ::"v"(seed)
      : CLOBBERS);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) body<OP>();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t r;
  asm volatile("v_bitop3_b32 %0, v20, v27, v35 bitop3:0x96" : "=v"(r)::CLOBBERS);
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

using Kfn = void (*)(unsigned long long*, uint32_t*, int);
#define KFN(n) k_valu<n>,
static const Kfn kKernels[] = {FOR_EACH_OP(KFN)};
#undef KFN

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const double clk_hz = prop.clockRate * 1e3;
  const int iters = 1024, max_b = 8;
  unsigned long long* cyc;
  uint32_t* out;
  CHECK(hipMalloc(&cyc, sizeof(unsigned long long) * cus * max_b));
  CHECK(hipMalloc(&out, sizeof(uint32_t) * 256 * cus * max_b));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::printf("{\"cus\": %d, \"clock_mhz\": %.0f, \"iters\": %d, \"results\": [\n", cus, clk_hz / 1e6, iters);
  bool first = true;
  for (int op = 0; op < kOps; ++op) {
    for (int b : {2, 4, 8}) {
      const int grid = cus * b;
      double best_ms = 1e30, best_cyc = 1e30;
      for (int rep = 0; rep < 4; ++rep) {
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(kKernels[op], dim3(grid), dim3(256), 0, 0, cyc, out, iters);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<unsigned long long> c(grid);
        CHECK(hipMemcpy(c.data(), cyc, sizeof(unsigned long long) * grid, hipMemcpyDeviceToHost));
        double mean = 0;
        for (auto v : c) mean += (double)v;
        mean /= grid;
        best_ms = std::min(best_ms, (double)ms);
        best_cyc = std::min(best_cyc, mean);
      }
      const double instr_per_wave = (double)iters * kBodyLen;
      const double cyc_per = best_cyc / (b * instr_per_wave);
      const double wall_per = best_ms * 1e-3 * clk_hz / (b * instr_per_wave);
      std::printf("%s {\"op\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_instr\": %.3f, \"wall_cyc_per_instr\": %.3f}",
                  first ? " " : ",\n ", kOpNames[op], b, cyc_per, wall_per);
      first = false;
    }
  }
  std::printf("\n]}\n");
  CHECK(hipFree(cyc));
  CHECK(hipFree(out));
  return 0;
}
