// Standalone timing of X11 stage-kernel variants against the production kernel (same inputs, outputs compared).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DOTEDAMA_X11_VARIANTS -Icsrc/include -Icsrc/kernels \
//          tools/x11_variants.hip -o tools/bin/x11_variants
// Run:   tools/bin/x11_variants [rounds]      -> one JSON line: ms per 2^23 nonces per variant (median of rounds)
//
// Each round launches every variant 10 times back to back (after a warm-up), rounds interleave the variants so
// clock drift hits all of them alike. A variant whose digests differ from the production kernel's is reported
// with "match": false.
#include "../csrc/kernels/x11_stages_a.hip"
#include "../csrc/kernels/x11_stages_b.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

using otedama::x11k::u32;
using otedama::x11k::u64;

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

__global__ void fill(u64* H, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    u64 x = i * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
    x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29;
    H[i] = x;
  }
}

// the production kernels take the batch's abort word: wrapped here without one (the variants have none)
namespace otedama::x11k {
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(7, 8))) void k_jh512_64_prod(
    u64* __restrict__ Hb, u32 stride, u32 n) {
  jh_stage_lds(Hb, stride, n, true);
}
__global__ __launch_bounds__(kAesBlock) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_shavite512_64_prod(
    u64* __restrict__ Hb, u32 stride, u32 n) {
  shavite_stage(Hb, stride, n, X11Abort{});
}
__global__ __launch_bounds__(kSimdBlock) void k_simd512_64_prod(u64* __restrict__ Hb, u32 stride, u32 n) {
  simd_stage<true>(Hb, stride, n);
}
}  // namespace otedama::x11k

typedef void (*StageFn)(u64*, u32, u32);
struct Variant {
  const char* name;
  StageFn fn;
  int kind;    // 0: one lane per nonce; 1: grid-stride AES-table kernel (512-thread blocks, 8 per CU);
               // 2: SIMD-512, eight lanes per nonce
  int group;   // variants of one stage share a group; outputs are compared with the group's first
};

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 3;
  const u32 n = 1u << 23, stride = n;
  const size_t words = 8ull * stride;
  u64 *src = nullptr, *H = nullptr;
  CK(hipMalloc(&src, words * 8));
  CK(hipMalloc(&H, words * 8));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, src, words);
  CK(hipGetLastError());
  using namespace otedama::x11k;
  std::vector<Variant> vs = {{"jh_lds_reload_w7 (production)", k_jh512_64_prod, 0, 0},
                             {"jh_sgpr", k_jh512_64_sgpr, 0, 0},
                             {"jh_lds_w7", k_jh512_64_w7, 0, 0},
                             {"jh_lds", k_jh512_64_lds, 0, 0},
                             {"shavite_4round_trips (production)", k_shavite512_64_prod, 1, 1},
                             {"shavite_r2 (round-2 kernel)", k_shavite512_64_r2, 1, 1},
                             {"simd_swizzle (production)", k_simd512_64_prod, 2, 2},
                             {"simd_dpp (round-2 lane exchange)", k_simd512_64_dpp, 2, 2}};
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  auto launch = [&](const Variant& v, u64* buf) {
    if (v.kind == 1) {
      const u32 want = (n + 511) / 512, cap = (u32)cus * 8;
      hipLaunchKernelGGL(v.fn, dim3(want < cap ? want : cap), dim3(512), 0, 0, buf, stride, n);
    } else if (v.kind == 2) {
      hipLaunchKernelGGL(v.fn, dim3(uint32_t((8ull * n + kBlock - 1) / kBlock)), dim3(kBlock), 0, 0, buf, stride, n);
    } else {
      hipLaunchKernelGGL(v.fn, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, 0, buf, stride, n);
    }
  };
  // reference digests: the first variant of each group
  std::vector<u64> a(words), b(words);
  std::vector<bool> match(vs.size(), true);
  for (size_t v = 0; v < vs.size(); ++v) {
    CK(hipMemcpy(H, src, words * 8, hipMemcpyDeviceToDevice));
    launch(vs[v], H);
    CK(hipDeviceSynchronize());
    if (v == 0 || vs[v].group != vs[v - 1].group) {
      CK(hipMemcpy(a.data(), H, words * 8, hipMemcpyDeviceToHost));
      continue;
    }
    CK(hipMemcpy(b.data(), H, words * 8, hipMemcpyDeviceToHost));
    match[v] = a == b;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ms(vs.size());
  for (int r = 0; r < rounds; ++r) {
    for (size_t v = 0; v < vs.size(); ++v) {
      CK(hipMemcpy(H, src, words * 8, hipMemcpyDeviceToDevice));
      launch(vs[v], H);  // warm-up (in place: inputs keep changing)
      CK(hipEventRecord(e0, 0));
      for (int k = 0; k < 10; ++k) launch(vs[v], H);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t / 10);
    }
  }
  std::printf("{\"n\": %u, \"rounds\": %d, \"variants\": {", n, rounds);
  for (size_t v = 0; v < vs.size(); ++v) {
    auto s = ms[v];
    std::sort(s.begin(), s.end());
    std::printf("%s\"%s\": {\"ms_median\": %.4f, \"ms\": [", v ? ", " : "", vs[v].name, s[s.size() / 2]);
    for (size_t k = 0; k < ms[v].size(); ++k) std::printf("%s%.4f", k ? ", " : "", ms[v][k]);
    std::printf("], \"match\": %s}", match[v] ? "true" : "false");
  }
  std::printf("}}\n");
  return 0;
}
