// libFuzzer harness (ASan + UBSan) for the native byte-parsing code ("fuzzing of the frame/JSON
// decoders ... libFuzzer on the C++ codec"; the reference fuzzes its Go decoder, stratum/frame_fuzz_test.go:25,85).
// Byte 0 of the input picks the target:
//   0: SV2 frame scanner (csrc/cpu/sv2_frame.cpp) vs a straight-line reference decoder; every record must match,
//      lie inside the buffer and tile it contiguously; the stop status must be explained by the next header.
//   1: SHA-256 / SHA-256d / X11 over arbitrary-length input (memory safety of the block loops and padding).
// Build/run: tools/sanitize/run.sh (target "fuzz"), or
//   clang++ -fsanitize=fuzzer,address,undefined -Icsrc/include tools/sanitize/fuzz_native.cpp csrc/cpu/sv2_frame.cpp \
//     csrc/cpu/sha256_cpu.cpp csrc/cpu/x11_cpu.cpp -o fuzz && ./fuzz -runs=200000
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "otedama/sha256.h"
#include "otedama/sv2_frame.h"
#include "otedama/x11.h"

using namespace otedama;

#define REQUIRE(c)                                                  \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "fuzz check failed: %s (line %d)\n", #c, __LINE__); \
      std::abort();                                                 \
    }                                                               \
  } while (0)

static void fuzz_sv2(const uint8_t* d, size_t n) {
  if (n < 2) return;
  // max frame between 6 bytes and 16 MiB, picked by the second byte
  const uint32_t max_frame = d[0] < 128 ? 6u + d[0] : (1u << 24);
  d += 1;
  n -= 1;
  std::vector<uint8_t> buf(d, d + n);  // exact-size heap copy: ASan sees any over-read
  const size_t cap = (size_t)(d[0] & 7) + 1;  // small caps exercise kSv2Full
  std::vector<Sv2FrameRec> recs(cap);
  size_t off = 0;
  while (true) {
    size_t consumed = 0;
    int status = -1;
    const size_t k = sv2_scan(buf.data() + off, buf.size() - off, max_frame, recs.data(), cap, &consumed, &status);
    REQUIRE(k <= cap && consumed <= buf.size() - off);
    size_t pos = 0;
    for (size_t i = 0; i < k; ++i) {  // reference decode of frame i
      const uint8_t* h = buf.data() + off + pos;
      const uint32_t ext = h[0] | (h[1] << 8), len = h[3] | (h[4] << 8) | ((uint32_t)h[5] << 16);
      REQUIRE(recs[i].extension_type == ext && recs[i].msg_type == h[2] && recs[i].length == len);
      REQUIRE(recs[i].offset == pos + kSv2HeaderSize);
      REQUIRE(kSv2HeaderSize + len <= max_frame);
      REQUIRE(!(ext & kSv2ChannelBit) || len >= kSv2MinChannelPayload);
      pos += kSv2HeaderSize + len;
    }
    REQUIRE(pos == consumed);
    const size_t rest = buf.size() - off - consumed;
    const uint8_t* h = buf.data() + off + consumed;
    if (status == kSv2Full) {
      REQUIRE(k == cap);
      off += consumed;
      continue;
    }
    if (status == kSv2Ok) {  // stopped at a partial header or partial frame
      if (rest >= kSv2HeaderSize) {
        const uint32_t len = h[3] | (h[4] << 8) | ((uint32_t)h[5] << 16);
        REQUIRE(kSv2HeaderSize + len > rest);
      }
    } else {
      REQUIRE(rest >= kSv2HeaderSize);
      const uint32_t ext = h[0] | (h[1] << 8), len = h[3] | (h[4] << 8) | ((uint32_t)h[5] << 16);
      if (status == kSv2TooLarge) REQUIRE((uint64_t)kSv2HeaderSize + len > max_frame);
      else REQUIRE(status == kSv2ShortChannel && (ext & kSv2ChannelBit) && len < kSv2MinChannelPayload);
    }
    break;
  }
}

static void fuzz_hashes(const uint8_t* d, size_t n) {
  std::vector<uint8_t> buf(d, d + n);
  uint8_t a[32], b[32], x[32];
  sha256(buf.data(), buf.size(), a);
  sha256d(buf.data(), buf.size(), b);
  sha256(a, 32, x);
  REQUIRE(std::memcmp(x, b, 32) == 0);  // sha256d == sha256(sha256)
  x11::x11(buf.data(), buf.size(), x, nullptr);
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size == 0) return 0;
  if ((data[0] & 1) == 0) fuzz_sv2(data + 1, size - 1);
  else fuzz_hashes(data + 1, size - 1);
  return 0;
}
