// SHA-256 host primitives shared by the CPU miner, the job precompute that feeds
// the gfx950 search kernels, share validation and the scrypt/PBKDF2 code.
//
// Parity: reference hot function is internal/miner/sha256d.go:107-117 (SHA256d,
// HashHeader). The reference re-serialises the 80-byte header and runs three
// full compressions per nonce; here the first 64 bytes are compressed once per
// job (midstate) and only block 2 + the digest block run per nonce.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>
#include <cstring>

namespace otedama {

extern const uint32_t kSha256K[64];
extern const uint32_t kSha256IV[8];

static inline uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static inline uint32_t load_be32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}
static inline uint32_t load_le32(const uint8_t* p) {
  return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}
static inline void store_be32(uint8_t* p, uint32_t v) {
  p[0] = uint8_t(v >> 24); p[1] = uint8_t(v >> 16); p[2] = uint8_t(v >> 8); p[3] = uint8_t(v);
}
static inline void store_le32(uint8_t* p, uint32_t v) {
  p[0] = uint8_t(v); p[1] = uint8_t(v >> 8); p[2] = uint8_t(v >> 16); p[3] = uint8_t(v >> 24);
}
static inline uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

// One SHA-256 compression of a 64-byte block into `state` (portable C++).
void sha256_compress_portable(uint32_t state[8], const uint8_t block[64]);
// Dispatches to SHA-NI when the CPU has it, else portable.
void sha256_compress(uint32_t state[8], const uint8_t block[64]);
// Two independent compressions, interleaved on SHA-NI (latency hiding); same results as two calls.
void sha256_compress_x2(uint32_t s0[8], const uint8_t b0[64], uint32_t s1[8], const uint8_t b1[64]);
// n independent compressions, interleaved in groups of up to 4 on SHA-NI (portable one by one otherwise).
void sha256_compress_xn(int n, uint32_t* const state[], const uint8_t* const block[]);
// SHA-NI nonce scan of an 80-byte header (midstate of block 1, tail12 = header bytes 64..75): appends the nonces of
// [start, start + done) whose H7 word passes the share filter (bswap(H7) <= thi; the caller re-verifies the full
// hash) and sets *done to the nonces covered (a multiple of `lanes`, 1..4). False without SHA-NI.
bool sha256d_scan_h7(int lanes, const uint32_t mid[8], const uint8_t tail12[12], uint32_t start, uint64_t count,
                     uint32_t thi, std::vector<uint32_t>* cands, uint64_t* done);
bool cpu_has_sha_ni();
// The same scan, 16 nonces per step on AVX-512 (F + BW); *done is a multiple of 16. False without AVX-512.
bool sha256d_scan_h7_wide(const uint32_t mid[8], const uint8_t tail12[12], uint32_t start, uint64_t count,
                          uint32_t thi, std::vector<uint32_t>* cands, uint64_t* done);
bool cpu_has_avx512_sha_scan();
int sha256d_scan_wide_groups();  // 16-lane groups in flight per step (OTEDAMA_CPU_SCAN_GROUPS, else by CPU vendor)

// Full SHA-256 of an arbitrary message.
void sha256(const uint8_t* data, size_t len, uint8_t out[32]);
// SHA-256(SHA-256(data)).
void sha256d(const uint8_t* data, size_t len, uint8_t out[32]);

// HMAC-SHA256 and PBKDF2-HMAC-SHA256 (used by scrypt's outer layers).
void hmac_sha256(const uint8_t* key, size_t klen, const uint8_t* msg, size_t mlen, uint8_t out[32]);
void pbkdf2_sha256(const uint8_t* pw, size_t pwlen, const uint8_t* salt, size_t saltlen,
                   uint32_t iters, uint8_t* out, size_t outlen);

// 256-bit little-endian compare (byte 31 most significant): a <= b.
static inline bool le256_leq(const uint8_t a[32], const uint8_t b[32]) {
  for (int i = 31; i >= 0; --i) {
    if (a[i] != b[i]) return a[i] < b[i];
  }
  return true;
}

}  // namespace otedama
