// SV2 frame-decode microbenchmark for the native scanner (csrc/cpu/sv2_frame.cpp).
//
// The reference quotes ~20 ns per header decode and ~200 ns per 1 KB full-frame decode (BENCHMARKS.md:68-69;
// its Go decoder reads one frame per call and allocates the payload). Here:
//   header : scan a buffer of empty-payload frames (6-byte headers only) -> ns per frame
//   full1k : scan 1 KiB-payload frames AND copy every payload into a fresh heap buffer -> ns per frame
// Build: g++ -O2 -std=c++17 -Icsrc/include tools/bench_sv2.cpp csrc/cpu/sv2_frame.cpp -o /tmp/bench_sv2
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>

#include "otedama/sv2_frame.h"

using namespace otedama;

static std::vector<uint8_t> make_stream(size_t frames, uint32_t payload) {
  std::vector<uint8_t> s;
  s.reserve(frames * (kSv2HeaderSize + payload));
  for (size_t i = 0; i < frames; ++i) {
    const uint16_t ext = (i & 1) ? 0x8000 : 0;
    const uint8_t hdr[6] = {(uint8_t)ext, (uint8_t)(ext >> 8), (uint8_t)(0x15 + (i & 7)), (uint8_t)payload,
                            (uint8_t)(payload >> 8), (uint8_t)(payload >> 16)};
    s.insert(s.end(), hdr, hdr + 6);
    for (uint32_t j = 0; j < payload; ++j) s.push_back((uint8_t)(i + j));
  }
  return s;
}

template <class F>
static double best_ns_per_frame(F&& body, size_t frames, int reps) {
  double best = 1e30;
  for (int r = 0; r < reps; ++r) {
    auto t0 = std::chrono::steady_clock::now();
    body();
    auto t1 = std::chrono::steady_clock::now();
    best = std::min(best, std::chrono::duration<double, std::nano>(t1 - t0).count() / (double)frames);
  }
  return best;
}

int main() {
  const size_t nh = 1 << 20, nf = 1 << 10, nf_iters = 64;  // 1 MiB of 1 KiB frames, cache-resident like a socket buffer
  auto hs = make_stream(nh, 4);  // 4-byte payload: the minimum a channel message may carry
  auto fs = make_stream(nf, 1024);
  std::vector<Sv2FrameRec> recs(nh);
  size_t consumed = 0, sink = 0;
  int status = 0;

  double h_ns = best_ns_per_frame([&] {
    size_t k = sv2_scan(hs.data(), hs.size(), 1u << 24, recs.data(), recs.size(), &consumed, &status);
    sink += k + recs[k - 1].length;
  }, nh, 20);
  if (consumed != hs.size() || status != kSv2Ok) return 1;

  double f_ns = best_ns_per_frame([&] {
    for (size_t it = 0; it < nf_iters; ++it) {
      size_t k = sv2_scan(fs.data(), fs.size(), 1u << 24, recs.data(), recs.size(), &consumed, &status);
      for (size_t i = 0; i < k; ++i) {  // own each payload, as a decoder returning frames must
        std::unique_ptr<uint8_t[]> p(new uint8_t[recs[i].length]);
        std::memcpy(p.get(), fs.data() + recs[i].offset, recs[i].length);
        sink += p[recs[i].length - 1];
      }
    }
  }, nf * nf_iters, 20);
  if (consumed != fs.size() || status != kSv2Ok) return 1;

  std::printf("{\"header_ns\": %.2f, \"header_frames_per_sec\": %.4g, \"full1k_ns\": %.2f, "
              "\"full1k_frames_per_sec\": %.4g, \"sink\": %zu}\n",
              h_ns, 1e9 / h_ns, f_ns, 1e9 / f_ns, sink);
  return 0;
}
