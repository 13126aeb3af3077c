// Same-process timing of the single-midstate SHA-256d search (BASELINE config 2) under its abort-poll forms.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/include -Icsrc/kernels \
//          -mllvm -pragma-unroll-threshold=1000000 tools/sha_single_ab.hip -o tools/bin/sha_single_ab
// Run:   tools/bin/sha_single_ab [rounds] [grid ...]   -> one JSON line per grid: GH/s per form (median of rounds)
//
// Forms: the production kernel (abort_peek right after the load), the split form of the multi-variant kernels
// (abort_issue / abort_seen; production here until profiles/r3/ad_single), and no poll at all; each with no abort
// word (the ops path, bench.py's single-midstate pass) and with an uncached abort word that never moves (the
// native miner). Every form must report the same hits.
#include "../csrc/kernels/sha256d_search.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      std::exit(1);                                                                           \
    }                                                                                         \
  } while (0)

using otedama_dev::abort_issue;
using otedama_dev::abort_newer;
using otedama_dev::abort_peek;
using otedama_dev::abort_seen;
using otedama_dev::hit_publish;

__global__ __launch_bounds__(256) void ab_single_split(const otedama::Sha256dParams p, uint32_t base, uint64_t count,
                                                       const otedama::HitSink sink) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t stride = gridDim.x * blockDim.x;
  uint32_t ab = abort_issue(sink), trip = 0;
  for (uint64_t off = tid; off < count; off += stride) {
    if (++trip == kAbortTrips) {
      if (abort_seen(ab, sink.epoch)) break;
      ab = abort_issue(sink);
      trip = 0;
    }
    const uint32_t nonce = base + static_cast<uint32_t>(off);
    const uint32_t h7 = sha256d_h7(p, __builtin_bswap32(nonce));
    if (__builtin_bswap32(h7) <= p.target_hi) hit_publish(sink, nonce, 0u);
  }
}

__global__ __launch_bounds__(256) void ab_single_nopoll(const otedama::Sha256dParams p, uint32_t base,
                                                        uint64_t count, const otedama::HitSink sink) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint64_t off = tid; off < count; off += stride) {
    const uint32_t nonce = base + static_cast<uint32_t>(off);
    const uint32_t h7 = sha256d_h7(p, __builtin_bswap32(nonce));
    if (__builtin_bswap32(h7) <= p.target_hi) hit_publish(sink, nonce, 0u);
  }
}

using Kern = void (*)(const otedama::Sha256dParams, uint32_t, uint64_t, const otedama::HitSink);

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
  std::vector<uint32_t> grids;
  for (int i = 2; i < argc; ++i) grids.push_back(uint32_t(std::atoi(argv[i])));
  if (grids.empty()) grids.push_back(1536);
  const uint64_t count = 1ull << 32;
  otedama::Sha256dParams p{};
  for (int i = 0; i < 8; ++i) p.mid[i] = 0x6a09e667u * (i + 3), p.st3[i] = 0x9e3779b9u * (i + 7);
  p.w0 = 0x01020304u, p.w1 = 0x5f5e1000u, p.w2 = 0x1d00ffffu, p.w16 = 0x11111111u, p.w17 = 0x22222222u;
  p.pre3 = 0x33333333u, p.t2_3 = 0x44444444u;
  p.target_hi = 0x00000fffu;  // ~1 candidate per 2^20 nonces: the hit path runs, the counts are compared

  const uint32_t cap = 1u << 14;
  uint32_t* out = nullptr;
  CK(hipMalloc(&out, (1 + cap) * sizeof(uint32_t)));
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
  std::vector<Form> forms = {{"prod_peek", otd_sha256d_search, false, {}},
                             {"split_issue_seen", ab_single_split, false, {}},
                             {"no_poll", ab_single_nopoll, false, {}},
                             {"prod_peek+word", otd_sha256d_search, true, {}},
                             {"split_issue_seen+word", ab_single_split, true, {}}};
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (const uint32_t grid : grids) {
  for (auto& f : forms) f.gh.clear(), f.hits = 0;
  for (auto& f : forms) {  // warm-up: load each code object once
    otedama::HitSink s;
    s.out = out, s.cap = cap, s.epoch = epoch, s.abort = f.word ? word : nullptr;
    hipLaunchKernelGGL(f.fn, dim3(grid), dim3(256), 0, 0, p, 0u, uint64_t(1) << 24, s);
  }
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r) {
    for (auto& f : forms) {
      otedama::HitSink s;
      s.out = out, s.cap = cap, s.epoch = epoch, s.abort = f.word ? word : nullptr;
      CK(hipMemset(out, 0, 4));
      CK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(f.fn, dim3(grid), dim3(256), 0, 0, p, 0u, count, s);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      f.gh.push_back(double(count) / (ms * 1e-3) / 1e9);
      uint32_t n = 0;
      CK(hipMemcpy(&n, out, 4, hipMemcpyDeviceToHost));
      if (r == 0) f.hits = n;
      else if (n != f.hits) std::fprintf(stderr, "%s: hit count changed %u -> %u\n", f.name, f.hits, n);
    }
  }
  std::printf("{\"grid\": %u, \"nonces\": %llu, \"rounds\": %d, \"forms\": {", grid, (unsigned long long)count, rounds);
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
