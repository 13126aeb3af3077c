// Same-process timing of the two-chain version-parallel SHA-256d kernel (bench.py's headline kernel,
// otd_sha256d_search_vn<2,0>) under its abort-poll forms: production (split issue/seen every trip), abort_peek every
// trip, and no poll; each with no abort word (the ops path, bench.py) and with an uncached abort word that never moves
// (the native miner). tools/sha_single_ab.hip does the same for the single-midstate kernel.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/include -Icsrc/kernels \
//          -mllvm -pragma-unroll-threshold=1000000 tools/sha_v_ab.hip -o tools/bin/sha_v_ab
// Run:   tools/bin/sha_v_ab [rounds] [blocks_per_cu ...]  -> one JSON line per grid: GH/s per form (median of rounds)
// Every form must report the same hits (synthetic variant table, target 2^-20).
#include "../csrc/kernels/sha256d_search_v.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      std::exit(1);                                                                           \
    }                                                                                         \
  } while (0)

template __global__ void otd_sha256d_search_vn<2, 0, 1>(const otedama::Sha256dParamsV, VarPtr, uint32_t, uint64_t,
                                                          const otedama::HitSink);
template __global__ void otd_sha256d_search_vn<2, 0, 2>(const otedama::Sha256dParamsV, VarPtr, uint32_t, uint64_t,
                                                          const otedama::HitSink);

using Kern = void (*)(const otedama::Sha256dParamsV, VarPtr, uint32_t, uint64_t, const otedama::HitSink);

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  std::vector<uint32_t> per_cu;
  for (int i = 2; i < argc; ++i) per_cu.push_back(uint32_t(std::atoi(argv[i])));
  if (per_cu.empty()) per_cu.push_back(128);  // ops/tuning.py SHA256D_V2_BLOCKS_PER_CU
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));

  // 128 variants (one two-chain group), 2^25 W3 values each: 2^32 hashes per launch, as the native miner issues them
  constexpr uint32_t kVars = 128;
  const uint64_t count = 1ull << 25;
  std::vector<otedama::Sha256dVariant> hv(kVars);
  uint32_t x = 0x12345678u;
  auto rnd = [&x]() { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; };
  for (auto& v : hv) {
    for (int i = 0; i < 8; ++i) v.mid[i] = rnd(), v.st3[i] = rnd();
    v.pre3 = rnd(), v.t2_3 = rnd();
  }
  otedama::Sha256dParamsV p{};
  p.w0 = 0x01020304u, p.w1 = 0x5f5e1000u, p.w2 = 0x1d00ffffu, p.w16 = 0x11111111u, p.w17 = 0x22222222u;
  p.target_hi = 0x00000fffu;
  p.groups = 1;  // groups of 64 * NC variants, as launch_sha256d_search_v passes them to the kernel
  otedama::Sha256dVariant* dv = nullptr;
  CK(hipMalloc(&dv, kVars * sizeof(otedama::Sha256dVariant)));
  CK(hipMemcpy(dv, hv.data(), kVars * sizeof(otedama::Sha256dVariant), hipMemcpyHostToDevice));
  const uint32_t cap = 1u << 14;
  uint32_t* out = nullptr;
  CK(hipMalloc(&out, (1 + 2 * cap) * sizeof(uint32_t)));
  uint32_t* word = nullptr;
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&word), 64, hipDeviceMallocUncached));
  const uint32_t epoch = 7;
  CK(hipMemcpy(word, &epoch, 4, hipMemcpyHostToDevice));

  struct Form {
    const char* name;
    Kern fn;
    bool word;
    std::vector<double> gh;
    uint32_t hits = 0;
  };
  std::vector<Form> forms = {{"prod_split", otd_sha256d_search_vn<2, 0, 0>, false, {}},
                             {"peek", otd_sha256d_search_vn<2, 0, 1>, false, {}},
                             {"no_poll", otd_sha256d_search_vn<2, 0, 2>, false, {}},
                             {"prod_split+word", otd_sha256d_search_vn<2, 0, 0>, true, {}},
                             {"peek+word", otd_sha256d_search_vn<2, 0, 1>, true, {}}};
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (const uint32_t pc : per_cu) {
    const uint32_t grid = uint32_t(cus) * pc;
    for (auto& f : forms) f.gh.clear(), f.hits = 0;
    for (auto& f : forms) {  // warm-up: load each code object once
      otedama::HitSink s;
      s.out = out, s.cap = cap, s.epoch = epoch, s.words = 2, s.abort = f.word ? word : nullptr;
      hipLaunchKernelGGL(f.fn, dim3(grid), dim3(256), 0, 0, p, dv, 0u, uint64_t(1) << 16, s);
    }
    CK(hipDeviceSynchronize());
    for (int r = 0; r < rounds; ++r) {
      for (auto& f : forms) {
        otedama::HitSink s;
        s.out = out, s.cap = cap, s.epoch = epoch, s.words = 2, s.abort = f.word ? word : nullptr;
        CK(hipMemset(out, 0, 4));
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(f.fn, dim3(grid), dim3(256), 0, 0, p, dv, 0u, count, s);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        f.gh.push_back(double(count) * kVars / (ms * 1e-3) / 1e9);
        uint32_t n = 0;
        CK(hipMemcpy(&n, out, 4, hipMemcpyDeviceToHost));
        if (r == 0) f.hits = n;
        else if (n != f.hits) std::fprintf(stderr, "%s: hit count changed %u -> %u\n", f.name, f.hits, n);
      }
    }
    std::printf("{\"blocks_per_cu\": %u, \"grid\": %u, \"hashes\": %llu, \"rounds\": %d, \"forms\": {", pc, grid,
                (unsigned long long)(count * kVars), rounds);
    for (size_t i = 0; i < forms.size(); ++i) {
      auto g = forms[i].gh;
      std::sort(g.begin(), g.end());
      std::printf("%s\"%s\": {\"ghs_median\": %.4f, \"ghs_min\": %.4f, \"ghs_max\": %.4f, \"hits\": %u, \"match\": %s}",
                  i ? ", " : "", forms[i].name, g[g.size() / 2], g.front(), g.back(), forms[i].hits,
                  forms[i].hits == forms[0].hits ? "true" : "false");
    }
    std::printf("}}\n");
    std::fflush(stdout);
  }
  return 0;
}
