// Stratum V2 frame scanner: splits a byte stream into frames without copying.
//
// Parity: internal/stratum/frame.go — 6-byte little-endian header (u16 extension_type with bit 15 = channel
// message, u8 msg_type, u24 msg_length; frame.go:57-86,172-186), header validation (channel payload >= 4 bytes,
// frame.go:108-136) and the max-frame-size check made BEFORE the payload is buffered (frame.go:285-293).
// The reference decodes one frame per blocking read; here a whole socket read is scanned in one native call and
// frames are handed out as (offset, length) views into the caller's buffer.
#pragma once
#include <cstddef>
#include <cstdint>

namespace otedama {

constexpr uint32_t kSv2HeaderSize = 6;
constexpr uint32_t kSv2ChannelBit = 0x8000;
constexpr uint32_t kSv2MinChannelPayload = 4;

struct Sv2FrameRec {
  uint32_t offset;          // payload offset in the scanned buffer
  uint32_t length;          // payload length (u24)
  uint16_t extension_type;  // raw, channel bit included
  uint8_t msg_type;
  uint8_t pad;
};

enum Sv2ScanStatus : int {
  kSv2Ok = 0,           // stopped at the end of the data or at a partial frame
  kSv2TooLarge = 1,     // header + payload exceeds max_frame (nothing past the bad header is read)
  kSv2ShortChannel = 2, // channel bit set with a payload shorter than 4 bytes
  kSv2Full = 3,         // `cap` records written; call again from *consumed
};

// Scans complete frames in buf[0, n). Writes at most `cap` records, sets *consumed to the byte offset just past
// the last complete frame returned and returns the number of records. *status says why scanning stopped; on an
// error *consumed points at the offending header.
size_t sv2_scan(const uint8_t* buf, size_t n, uint32_t max_frame, Sv2FrameRec* out, size_t cap, size_t* consumed,
                int* status);

}  // namespace otedama
