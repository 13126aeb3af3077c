// Job parameter blocks handed from the host runtime to the gfx950 search kernels.
//
// Everything that does not depend on the nonce is folded on the host once per
// job variant (midstate of block 1, rounds 0..2 of block 2, W16/W17), so the
// per-nonce work on the GPU starts at round 3 with the nonce as W3. The
// reference hashes the whole 80-byte header per nonce with no midstate
// (internal/miner/sha256d.go:114-117, worker.go:250-280).
#pragma once
#include <cstdint>

namespace otedama {

// Kernel argument block for sha256d_search (passed by value -> SGPRs).
struct Sha256dParams {
  uint32_t mid[8];     // SHA-256 state after block 1 (header bytes 0..63)
  uint32_t st3[8];     // a..h of block 2 after rounds 0..2
  uint32_t w0, w1, w2; // block-2 words: merkle tail, ntime, nbits (big-endian loads)
  uint32_t w16, w17;   // nonce-independent schedule words
  uint32_t pre3;       // round-3 T1 without the nonce: h + S1(e) + Ch(e,f,g) + K3
  uint32_t t2_3;       // round-3 T2: S0(a) + Maj(a,b,c)
  uint32_t target_hi;  // most-significant 32 bits of the LE share target (bytes 28..31)
};

// Builds the kernel parameter block from an 80-byte header (nonce bytes ignored)
// and a 32-byte little-endian target.
void sha256d_prepare(const uint8_t header80[80], const uint8_t target32[32], Sha256dParams* out);

// K (2..16) header variants with identical bytes 64..79 (block 2 of the first hash: merkle tail,
// ntime, nbits, nonce) and different block 1 (BIP320 version rolling): one shared block-2 message
// schedule per nonce, K midstates (sha256d_search_k).
constexpr int kSha256dMaxK = 16;
// The K values sha256d_search_k is instantiated for; sha256d_k_floor(k) is the largest one <= k (1 if k < 2).
constexpr int sha256d_k_floor(int k) {
  return k >= 16 ? 16 : k >= 12 ? 12 : k >= 8 ? 8 : k >= 6 ? 6 : k >= 4 ? 4 : k >= 3 ? 3 : k >= 2 ? 2 : 1;
}
struct Sha256dVariant {
  uint32_t mid[8];
  uint32_t st3[8];
  uint32_t pre3, t2_3;
};
struct Sha256dParamsK {
  uint32_t w0, w1, w2, w16, w17;
  uint32_t target_hi;
  int32_t k;
  Sha256dVariant var[kSha256dMaxK];
};
// Returns false (and leaves *out undefined) unless k is an instantiated K (sha256d_k_floor(k) == k) and every header has the
// same bytes 64..75.
bool sha256d_prepare_k(const uint8_t* const headers80[], int k, const uint8_t target32[32], Sha256dParamsK* out);

// Version-parallel search (sha256d_search_v): 64 * groups variants with identical bytes 64..75, one per lane;
// the per-variant blocks live in device memory (vars[64 * groups]), the shared block-2 words in the kernarg.
constexpr int kSha256dVGroup = 64;  // variants per wave (wave64 lanes)
constexpr int kSha256dV2Group = 128;  // two-chain version-parallel kernel: two variants per lane
struct Sha256dParamsV {
  uint32_t w0, w1, w2, w16, w17;
  uint32_t target_hi;
  uint32_t groups;  // variant groups of 64
  uint32_t occupancy8;  // launch the 8-waves/SIMD build (launch-time choice, not part of the job)
};
// Fills *p and vars[0..n) (n a positive multiple of 64); false unless every header has the same bytes 64..75.
bool sha256d_prepare_v(const uint8_t* const headers80[], int n, const uint8_t target32[32], Sha256dParamsV* p,
                       Sha256dVariant* vars);

// Scrypt (N, r=1, p=1) job parameters: the 76-byte header prefix; the nonce is
// appended per lane as bytes 76..79.
// The HMAC key is the whole 80-byte header (> 64 B, so K' = SHA-256(header)),
// which contains the nonce: only SHA-256 of the first 64 header bytes (hmid) is
// nonce-independent; the PBKDF2 layers run per lane.
struct ScryptParams {
  uint32_t hdr[19];    // header words 0..18 as little-endian loads (bytes 0..75)
  uint32_t hmid[8];    // SHA-256 state after header bytes 0..63
  uint32_t target_hi;  // most-significant 32 bits of the LE share target
};

void scrypt_prepare(const uint8_t header80[80], const uint8_t target32[32], ScryptParams* out);

// X11 (Dash) job parameters. Stage 1 (BLAKE-512) sees the whole 80-byte header
// as one padded block; only the low half of message word 9 carries the nonce.
struct X11Params {
  uint64_t m[9];       // header bytes 0..71 as big-endian 64-bit words
  uint64_t m9_hi;      // header bytes 72..75 (nbits) in the high half of word 9
  uint64_t target_hi;  // most-significant 64 bits of the LE share target (bytes 24..31)
};

void x11_prepare(const uint8_t header80[80], const uint8_t target32[32], X11Params* out);

// `gap` selector for launch_scrypt_search: 1/2/4 = per-lane ROMix with that lookup gap,
// kScryptCoop = lane-cooperative ROMix (full-line octet lookups, gap 1).
constexpr int kScryptCoop = 8;
constexpr int kScryptLaneW8 = 9;   // per-lane ROMix, gap 1, pinned to 8 waves/SIMD
constexpr int kScryptCoop2 = 11;   // cooperative ROMix, two software-pipelined hashes per lane (gap 1)
constexpr int kScryptCoopSplit = 12;  // cooperative ROMix, write and lookup phases as two launches (gap 1)

}  // namespace otedama
