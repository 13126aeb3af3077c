// Stratum V2 frame scanner (see otedama/sv2_frame.h; reference internal/stratum/frame.go:238-302).
#include "otedama/sv2_frame.h"

#include <cstring>

namespace otedama {

size_t sv2_scan(const uint8_t* buf, size_t n, uint32_t max_frame, Sv2FrameRec* out, size_t cap, size_t* consumed,
                int* status) {
  size_t off = 0, k = 0;
  *status = kSv2Ok;
  while (n - off >= kSv2HeaderSize) {
    if (k == cap) {
      *status = kSv2Full;
      break;
    }
    uint64_t h = 0;
    if (n - off >= 8) {
      std::memcpy(&h, buf + off, 8);  // one unaligned load; the two bytes past the header are ignored
    } else {
      std::memcpy(&h, buf + off, kSv2HeaderSize);
    }
    const uint32_t ext = (uint32_t)(h & 0xFFFF);
    const uint32_t len = (uint32_t)(h >> 24) & 0xFFFFFF;
    if ((uint64_t)kSv2HeaderSize + len > max_frame) {
      *status = kSv2TooLarge;
      break;
    }
    if ((ext & kSv2ChannelBit) && len < kSv2MinChannelPayload) {
      *status = kSv2ShortChannel;
      break;
    }
    const size_t end = off + kSv2HeaderSize + len;
    if (end > n) break;  // partial frame: wait for more bytes
    Sv2FrameRec& r = out[k++];
    r.offset = (uint32_t)(off + kSv2HeaderSize);
    r.length = len;
    r.extension_type = (uint16_t)ext;
    r.msg_type = (uint8_t)(h >> 16);
    r.pad = 0;
    off = end;
  }
  *consumed = off;
  return k;
}

}  // namespace otedama
