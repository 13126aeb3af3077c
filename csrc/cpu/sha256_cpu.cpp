// Host SHA-256: portable C++ compression plus an x86 SHA-NI path.
//
// The SHA-NI path is the CPU baseline of BASELINE.json config 1 ("SHA-256d
// single-thread CPU miner"), which the reference gets from Go's stdlib assembly
// (internal/miner/sha256d.go:13-20). It is selected at run time via CPUID.
#include "otedama/sha256.h"

#include <cpuid.h>
#include <cstdlib>
#include <cstring>
#include <immintrin.h>

#include <type_traits>
#include <vector>

namespace otedama {

const uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

const uint32_t kSha256IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                               0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

void sha256_compress_portable(uint32_t state[8], const uint8_t block[64]) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i) w[i] = load_be32(block + 4 * i);
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = state[0], b = state[1], c = state[2], d = state[3];
  uint32_t e = state[4], f = state[5], g = state[6], h = state[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + kSha256K[i] + w[i];
    uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  state[0] += a; state[1] += b; state[2] += c; state[3] += d;
  state[4] += e; state[5] += f; state[6] += g; state[7] += h;
}

// SHA-NI compression (Intel SHA extensions). Standard message-schedule
// pipelining with sha256msg1/msg2 and two rounds per sha256rnds2.
__attribute__((target("sha,sse4.1")))
static void sha256_compress_shani(uint32_t state[8], const uint8_t block[64]) {
  const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i TMP = _mm_loadu_si128((const __m128i*)&state[0]);
  __m128i STATE1 = _mm_loadu_si128((const __m128i*)&state[4]);
  TMP = _mm_shuffle_epi32(TMP, 0xB1);          // CDAB
  STATE1 = _mm_shuffle_epi32(STATE1, 0x1B);    // EFGH
  __m128i STATE0 = _mm_alignr_epi8(TMP, STATE1, 8);  // ABEF
  STATE1 = _mm_blend_epi16(STATE1, TMP, 0xF0);       // CDGH
  const __m128i ABEF_SAVE = STATE0, CDGH_SAVE = STATE1;

  __m128i MSG, MSG0, MSG1, MSG2, MSG3;
  const __m128i* K = (const __m128i*)kSha256K;

  MSG0 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(block + 0)), MASK);
  MSG1 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(block + 16)), MASK);
  MSG2 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(block + 32)), MASK);
  MSG3 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(block + 48)), MASK);

#define QROUND(Mi, k)                                              \
  MSG = _mm_add_epi32(Mi, _mm_loadu_si128(K + (k)));               \
  STATE1 = _mm_sha256rnds2_epu32(STATE1, STATE0, MSG);             \
  MSG = _mm_shuffle_epi32(MSG, 0x0E);                              \
  STATE0 = _mm_sha256rnds2_epu32(STATE0, STATE1, MSG);

  // Rounds 0..15
  QROUND(MSG0, 0);
  QROUND(MSG1, 1); MSG0 = _mm_sha256msg1_epu32(MSG0, MSG1);
  QROUND(MSG2, 2); MSG1 = _mm_sha256msg1_epu32(MSG1, MSG2);
  QROUND(MSG3, 3);
  // Rounds 16..63: schedule W[t] for the next group while hashing this one.
  for (int k = 4; k < 16; k += 4) {
    TMP = _mm_alignr_epi8(MSG3, MSG2, 4); MSG0 = _mm_add_epi32(MSG0, TMP);
    MSG0 = _mm_sha256msg2_epu32(MSG0, MSG3); MSG2 = _mm_sha256msg1_epu32(MSG2, MSG3);
    QROUND(MSG0, k);
    TMP = _mm_alignr_epi8(MSG0, MSG3, 4); MSG1 = _mm_add_epi32(MSG1, TMP);
    MSG1 = _mm_sha256msg2_epu32(MSG1, MSG0); MSG3 = _mm_sha256msg1_epu32(MSG3, MSG0);
    QROUND(MSG1, k + 1);
    TMP = _mm_alignr_epi8(MSG1, MSG0, 4); MSG2 = _mm_add_epi32(MSG2, TMP);
    MSG2 = _mm_sha256msg2_epu32(MSG2, MSG1); MSG0 = _mm_sha256msg1_epu32(MSG0, MSG1);
    QROUND(MSG2, k + 2);
    TMP = _mm_alignr_epi8(MSG2, MSG1, 4); MSG3 = _mm_add_epi32(MSG3, TMP);
    MSG3 = _mm_sha256msg2_epu32(MSG3, MSG2); MSG1 = _mm_sha256msg1_epu32(MSG1, MSG2);
    QROUND(MSG3, k + 3);
  }
#undef QROUND

  STATE0 = _mm_add_epi32(STATE0, ABEF_SAVE);
  STATE1 = _mm_add_epi32(STATE1, CDGH_SAVE);
  TMP = _mm_shuffle_epi32(STATE0, 0x1B);            // FEBA
  STATE1 = _mm_shuffle_epi32(STATE1, 0xB1);         // DCHG
  STATE0 = _mm_blend_epi16(TMP, STATE1, 0xF0);      // DCBA
  STATE1 = _mm_alignr_epi8(STATE1, TMP, 8);         // ABEF -> HGFE
  _mm_storeu_si128((__m128i*)&state[0], STATE0);
  _mm_storeu_si128((__m128i*)&state[4], STATE1);
}

// N independent compressions interleaved (N = 2): sha256rnds2 is latency-bound in a single chain
// (each pair of rounds depends on the previous one), so two nonces in flight roughly double the
// per-core SHA-256d rate of the CPU miner. Same schedule as sha256_compress_shani, per lane.
template <int N>
__attribute__((target("sha,sse4.1"))) static void sha256_compress_shani_xn(uint32_t* const state[N],
                                                                          const uint8_t* const block[N]) {
  const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  const __m128i* K = (const __m128i*)kSha256K;
  __m128i S0[N], S1[N], A0[N], A1[N], M0[N], M1[N], M2[N], M3[N], MSG[N], TMP[N];
  for (int l = 0; l < N; ++l) {
    TMP[l] = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&state[l][0]), 0xB1);
    S1[l] = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&state[l][4]), 0x1B);
    S0[l] = _mm_alignr_epi8(TMP[l], S1[l], 8);
    S1[l] = _mm_blend_epi16(S1[l], TMP[l], 0xF0);
    A0[l] = S0[l]; A1[l] = S1[l];
    M0[l] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(block[l] + 0)), MASK);
    M1[l] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(block[l] + 16)), MASK);
    M2[l] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(block[l] + 32)), MASK);
    M3[l] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(block[l] + 48)), MASK);
  }
#define QR(Mi, k)                                                    \
  for (int l = 0; l < N; ++l) {                                      \
    MSG[l] = _mm_add_epi32(Mi[l], _mm_loadu_si128(K + (k)));         \
    S1[l] = _mm_sha256rnds2_epu32(S1[l], S0[l], MSG[l]);             \
    MSG[l] = _mm_shuffle_epi32(MSG[l], 0x0E);                        \
    S0[l] = _mm_sha256rnds2_epu32(S0[l], S1[l], MSG[l]);             \
  }
#define SCHED(Ma, Mb, Mc, Md)                                         \
  for (int l = 0; l < N; ++l) {                                       \
    TMP[l] = _mm_alignr_epi8(Md[l], Mc[l], 4); Ma[l] = _mm_add_epi32(Ma[l], TMP[l]); \
    Ma[l] = _mm_sha256msg2_epu32(Ma[l], Md[l]); Mc[l] = _mm_sha256msg1_epu32(Mc[l], Md[l]); \
  }
  QR(M0, 0);
  QR(M1, 1); for (int l = 0; l < N; ++l) M0[l] = _mm_sha256msg1_epu32(M0[l], M1[l]);
  QR(M2, 2); for (int l = 0; l < N; ++l) M1[l] = _mm_sha256msg1_epu32(M1[l], M2[l]);
  QR(M3, 3);
  for (int k = 4; k < 16; k += 4) {
    SCHED(M0, M1, M2, M3); QR(M0, k);
    SCHED(M1, M2, M3, M0); QR(M1, k + 1);
    SCHED(M2, M3, M0, M1); QR(M2, k + 2);
    SCHED(M3, M0, M1, M2); QR(M3, k + 3);
  }
#undef QR
#undef SCHED
  for (int l = 0; l < N; ++l) {
    S0[l] = _mm_add_epi32(S0[l], A0[l]);
    S1[l] = _mm_add_epi32(S1[l], A1[l]);
    TMP[l] = _mm_shuffle_epi32(S0[l], 0x1B);
    S1[l] = _mm_shuffle_epi32(S1[l], 0xB1);
    S0[l] = _mm_blend_epi16(TMP[l], S1[l], 0xF0);
    S1[l] = _mm_alignr_epi8(S1[l], TMP[l], 8);
    _mm_storeu_si128((__m128i*)&state[l][0], S0[l]);
    _mm_storeu_si128((__m128i*)&state[l][4], S1[l]);
  }
}

// SHA-256d of L consecutive nonces of one 80-byte header, up to the word the share filter needs (H7), on SHA-NI.
// Specialised for mining: rounds 0-1 of the header's second block use only W0, W1 (no nonce) and are hashed once
// per call (s1_pre); the first hash's state goes to the second block's message registers directly (no store,
// byte swap and reload); the second hash stops after round 61, where the F lane of the ABEF register already holds
// e61 = h64, so H7 = F + IV7 (rounds 62-63 and the feed-forward of the other words are skipped).
template <int L>
__attribute__((target("sha,sse4.1"))) static void sha256d_h7_shani(__m128i abef_mid, __m128i cdgh_mid, __m128i s1_pre,
                                                                  __m128i m0_tmpl, uint32_t nonce0, uint32_t h7[L]) {
  const __m128i* K = (const __m128i*)kSha256K;
  const __m128i PAD1 = _mm_set_epi32(0, 0, 0, int(0x80000000u));  // W4 = 0x80000000 (dword 0), W5..W7 = 0
  const __m128i LEN1 = _mm_set_epi32(640, 0, 0, 0);               // W15 = 640 bits
  const __m128i LEN2 = _mm_set_epi32(256, 0, 0, 0);               // second block: W15 = 256 bits
  const __m128i IV_ABEF = _mm_set_epi32(int(0x6a09e667u), int(0xbb67ae85u), int(0x510e527fu), int(0x9b05688cu));
  const __m128i IV_CDGH = _mm_set_epi32(int(0x3c6ef372u), int(0xa54ff53au), int(0x1f83d9abu), int(0x5be0cd19u));
  __m128i S0[L], S1[L], M0[L], M1[L], M2[L], M3[L], MSG[L], TMP[L];
#define QR(Mi, k)                                                    \
  for (int l = 0; l < L; ++l) {                                      \
    MSG[l] = _mm_add_epi32(Mi[l], _mm_loadu_si128(K + (k)));         \
    S1[l] = _mm_sha256rnds2_epu32(S1[l], S0[l], MSG[l]);             \
    MSG[l] = _mm_shuffle_epi32(MSG[l], 0x0E);                        \
    S0[l] = _mm_sha256rnds2_epu32(S0[l], S1[l], MSG[l]);             \
  }
#define SCHED(Ma, Mb, Mc, Md)                                         \
  for (int l = 0; l < L; ++l) {                                       \
    TMP[l] = _mm_alignr_epi8(Md[l], Mc[l], 4); Ma[l] = _mm_add_epi32(Ma[l], TMP[l]); \
    Ma[l] = _mm_sha256msg2_epu32(Ma[l], Md[l]); Mc[l] = _mm_sha256msg1_epu32(Mc[l], Md[l]); \
  }
  // ---- first hash, block 2 (from the midstate); rounds 0-1 are s1_pre
  for (int l = 0; l < L; ++l) {
    M0[l] = _mm_insert_epi32(m0_tmpl, int(__builtin_bswap32(nonce0 + uint32_t(l))), 3);  // W3: nonce bytes, BE
    M1[l] = PAD1;
    M2[l] = _mm_setzero_si128();
    M3[l] = LEN1;
    MSG[l] = _mm_shuffle_epi32(_mm_add_epi32(M0[l], _mm_loadu_si128(K)), 0x0E);
    S1[l] = s1_pre;
    S0[l] = _mm_sha256rnds2_epu32(abef_mid, s1_pre, MSG[l]);  // rounds 2-3 (W2, W3 = nonce)
  }
  QR(M1, 1); for (int l = 0; l < L; ++l) M0[l] = _mm_sha256msg1_epu32(M0[l], M1[l]);
  QR(M2, 2); for (int l = 0; l < L; ++l) M1[l] = _mm_sha256msg1_epu32(M1[l], M2[l]);
  QR(M3, 3);
  for (int k = 4; k < 16; k += 4) {
    SCHED(M0, M1, M2, M3); QR(M0, k);
    SCHED(M1, M2, M3, M0); QR(M1, k + 1);
    SCHED(M2, M3, M0, M1); QR(M2, k + 2);
    SCHED(M3, M0, M1, M2); QR(M3, k + 3);
  }
  // feed-forward, then the digest words straight into the second block's message registers (dword 0 = H0 / H4)
  for (int l = 0; l < L; ++l) {
    S0[l] = _mm_add_epi32(S0[l], abef_mid);
    S1[l] = _mm_add_epi32(S1[l], cdgh_mid);
    TMP[l] = _mm_shuffle_epi32(S0[l], 0x1B);
    S1[l] = _mm_shuffle_epi32(S1[l], 0xB1);
    M0[l] = _mm_blend_epi16(TMP[l], S1[l], 0xF0);
    M1[l] = _mm_alignr_epi8(S1[l], TMP[l], 8);
    M2[l] = PAD1;
    M3[l] = LEN2;
    S0[l] = IV_ABEF;
    S1[l] = IV_CDGH;
  }
  // ---- second hash, rounds 0..61
  QR(M0, 0);
  QR(M1, 1); for (int l = 0; l < L; ++l) M0[l] = _mm_sha256msg1_epu32(M0[l], M1[l]);
  QR(M2, 2); for (int l = 0; l < L; ++l) M1[l] = _mm_sha256msg1_epu32(M1[l], M2[l]);
  QR(M3, 3);
  for (int k = 4; k < 12; k += 4) {
    SCHED(M0, M1, M2, M3); QR(M0, k);
    SCHED(M1, M2, M3, M0); QR(M1, k + 1);
    SCHED(M2, M3, M0, M1); QR(M2, k + 2);
    SCHED(M3, M0, M1, M2); QR(M3, k + 3);
  }
  SCHED(M0, M1, M2, M3); QR(M0, 12);
  SCHED(M1, M2, M3, M0); QR(M1, 13);
  SCHED(M2, M3, M0, M1); QR(M2, 14);
  for (int l = 0; l < L; ++l) {  // W60..W63, then rounds 60-61 only
    TMP[l] = _mm_alignr_epi8(M2[l], M1[l], 4); M3[l] = _mm_add_epi32(M3[l], TMP[l]);
    M3[l] = _mm_sha256msg2_epu32(M3[l], M2[l]);
    MSG[l] = _mm_add_epi32(M3[l], _mm_loadu_si128(K + 15));
    S1[l] = _mm_sha256rnds2_epu32(S1[l], S0[l], MSG[l]);
    h7[l] = uint32_t(_mm_cvtsi128_si32(S1[l])) + 0x5be0cd19u;  // F lane of ABEF after round 61 = h64
  }
#undef QR
#undef SCHED
}

__attribute__((target("sha,sse4.1"))) static void sha256d_scan_h7_shani(int lanes, const uint32_t mid[8],
                                                                       const uint8_t tail12[12], uint32_t start,
                                                                       uint64_t count, uint32_t thi,
                                                                       std::vector<uint32_t>* cands,
                                                                       uint64_t* done) {
  __m128i TMP = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&mid[0]), 0xB1);
  __m128i CDGH = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&mid[4]), 0x1B);
  const __m128i ABEF = _mm_alignr_epi8(TMP, CDGH, 8);
  CDGH = _mm_blend_epi16(CDGH, TMP, 0xF0);
  const __m128i m0 = _mm_set_epi32(0, int(load_be32(tail12 + 8)), int(load_be32(tail12 + 4)), int(load_be32(tail12)));
  const __m128i s1_pre = _mm_sha256rnds2_epu32(CDGH, ABEF, _mm_add_epi32(m0, _mm_loadu_si128((const __m128i*)kSha256K)));
  uint32_t h7[4];
  uint64_t i = 0;
  auto scan = [&](auto lanes_c) {
    constexpr int Lc = decltype(lanes_c)::value;
    for (; i + Lc <= count; i += Lc) {
      const uint32_t n0 = start + uint32_t(i);
      sha256d_h7_shani<Lc>(ABEF, CDGH, s1_pre, m0, n0, h7);
      for (int l = 0; l < Lc; ++l)
        if (__builtin_bswap32(h7[l]) <= thi) cands->push_back(n0 + uint32_t(l));
    }
  };
  switch (lanes) {
    case 1: scan(std::integral_constant<int, 1>{}); break;
    case 2: scan(std::integral_constant<int, 2>{}); break;
    case 3: scan(std::integral_constant<int, 3>{}); break;
    default: scan(std::integral_constant<int, 4>{}); break;
  }
  *done = i;
}

// The same H7 scan for 16 nonces per step on AVX-512: one nonce per 32-bit lane, the eight working variables in
// zmm registers, Ch / Maj / the three-rotate sums as single vpternlogd, rotates as vprord. What does not depend on
// the nonce is hoisted out of the loop: rounds 0-2 of the first hash (W0-W2 come from the header), and the message
// words W16, W17 of the first hash; the zero and padding words of both blocks are compile-time constants, so their
// schedule terms fold away. The second hash stops at e61 = h64 as the SHA-NI scan does.
#define ZROR(x, n) _mm512_ror_epi32((x), (n))
#define ZS0(x) _mm512_ternarylogic_epi32(ZROR(x, 2), ZROR(x, 13), ZROR(x, 22), 0x96)
#define ZS1(x) _mm512_ternarylogic_epi32(ZROR(x, 6), ZROR(x, 11), ZROR(x, 25), 0x96)
#define Zs0(x) _mm512_ternarylogic_epi32(ZROR(x, 7), ZROR(x, 18), _mm512_srli_epi32((x), 3), 0x96)
#define Zs1(x) _mm512_ternarylogic_epi32(ZROR(x, 17), ZROR(x, 19), _mm512_srli_epi32((x), 10), 0x96)
#define ZCH(e, f, g) _mm512_ternarylogic_epi32((e), (f), (g), 0xCA)
#define ZMAJ(a, b, c) _mm512_ternarylogic_epi32((a), (b), (c), 0xE8)
#define ZADD(x, y) _mm512_add_epi32((x), (y))
#define ZC(x) _mm512_set1_epi32(int(x))
// one round on each of G independent groups (G chains in flight hide the round's dependency latency); kw(g) is
// K[t] + W[t] of group g
#define ZROUND(a, b, c, d, e, f, g, h, kw)                                         \
  for (int q = 0; q < G; ++q) {                                                    \
    const __m512i t1 = ZADD(ZADD(h[q], ZS1(e[q])), ZADD(ZCH(e[q], f[q], g[q]), (kw))); \
    d[q] = ZADD(d[q], t1);                                                         \
    h[q] = ZADD(t1, ZADD(ZS0(a[q]), ZMAJ(a[q], b[q], c[q])));                      \
  }

struct ScanPre {  // per header: the scalar prologue shared by every step
  uint32_t w0, w1, w2, w16, w17;
  uint32_t st[8];  // block-2 state after rounds 0-2
  // nonce-free parts of the first hash's schedule (W3 = nonce, W4 = 0x80000000, W5..W14 = 0, W15 = 640)
  uint32_t c18, c19, c30, c31, c32;
  uint32_t r3_t1, r3_t2;  // round 3: T1 without K3 + W3, and T2 (the state after round 2 is nonce-free)
  // the second hash's constants (X8 = 0x80000000, X9..X14 = 0, X15 = 256; round 0 on the IV)
  uint32_t x17, x23, x30, r0_t1, r0_t2;
};

// G x 16 consecutive nonces from n0: pushes those whose bswap(H7) <= thi
template <int G>
__attribute__((target("avx512f,avx512bw"))) static inline void sha256d_h7_x16(const ScanPre& p, const uint32_t mid[8],
                                                                          uint32_t n0, uint32_t thi,
                                                                          std::vector<uint32_t>* cands) {
  const __m512i bswap = _mm512_set4_epi32(0x0c0d0e0f, 0x08090a0b, 0x04050607, 0x00010203);
  const __m512i lane = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  // ---- first hash, block 2: W3 = the nonce's header bytes read big-endian
  __m512i W[G][64];
  __m512i a[G], b[G], c[G], d[G], e[G], f[G], g[G], h[G];
  for (int q = 0; q < G; ++q) {
    W[q][3] = _mm512_shuffle_epi8(ZADD(ZC(n0 + 16u * uint32_t(q)), lane), bswap);
    W[q][0] = ZC(p.w0); W[q][1] = ZC(p.w1); W[q][2] = ZC(p.w2); W[q][4] = ZC(0x80000000u);
    for (int t = 5; t < 15; ++t) W[q][t] = ZC(0);
    W[q][15] = ZC(640);
    W[q][16] = ZC(p.w16);
    W[q][17] = ZC(p.w17);
    a[q] = ZC(p.st[0]); b[q] = ZC(p.st[1]); c[q] = ZC(p.st[2]); d[q] = ZC(p.st[3]);
    e[q] = ZC(p.st[4]); f[q] = ZC(p.st[5]); g[q] = ZC(p.st[6]); h[q] = ZC(p.st[7]);
  }
  for (int q = 0; q < G; ++q) {  // W18..W32: the terms on the constant words W4..W17 are scalars (ScanPre)
    __m512i* w = W[q];
    w[18] = ZADD(ZC(p.c18), Zs0(w[3]));
    w[19] = ZADD(ZC(p.c19), w[3]);
    w[20] = ZADD(Zs1(w[18]), ZC(0x80000000u));
    w[21] = Zs1(w[19]);
    w[22] = ZADD(Zs1(w[20]), ZC(640));
    w[23] = ZADD(Zs1(w[21]), ZC(p.w16));
    w[24] = ZADD(Zs1(w[22]), ZC(p.w17));
    for (int t = 25; t < 30; ++t) w[t] = ZADD(Zs1(w[t - 2]), w[t - 7]);
    w[30] = ZADD(ZADD(Zs1(w[28]), w[23]), ZC(p.c30));
    w[31] = ZADD(ZADD(Zs1(w[29]), w[24]), ZC(p.c31));
    w[32] = ZADD(ZADD(Zs1(w[30]), w[25]), ZC(p.c32));
  }
#pragma GCC unroll 64
  for (int t = 33; t < 64; ++t)
    for (int q = 0; q < G; ++q)
      W[q][t] = ZADD(ZADD(Zs1(W[q][t - 2]), W[q][t - 7]), ZADD(Zs0(W[q][t - 15]), W[q][t - 16]));
  for (int q = 0; q < G; ++q) {  // round 3: everything but K3 + W3 is nonce-free
    const __m512i t1 = ZADD(ZC(p.r3_t1 + kSha256K[3]), W[q][3]);
    d[q] = ZADD(d[q], t1);
    h[q] = ZADD(t1, ZC(p.r3_t2));
  }
#pragma GCC unroll 64
  for (int t = 3; t < 64; t += 8) {
    if (t != 3) ZROUND(a, b, c, d, e, f, g, h, ZADD(ZC(kSha256K[t]), W[q][t]));
    if (t + 1 < 64) ZROUND(h, a, b, c, d, e, f, g, ZADD(ZC(kSha256K[t + 1]), W[q][t + 1]));
    if (t + 2 < 64) ZROUND(g, h, a, b, c, d, e, f, ZADD(ZC(kSha256K[t + 2]), W[q][t + 2]));
    if (t + 3 < 64) ZROUND(f, g, h, a, b, c, d, e, ZADD(ZC(kSha256K[t + 3]), W[q][t + 3]));
    if (t + 4 < 64) ZROUND(e, f, g, h, a, b, c, d, ZADD(ZC(kSha256K[t + 4]), W[q][t + 4]));
    if (t + 5 < 64) ZROUND(d, e, f, g, h, a, b, c, ZADD(ZC(kSha256K[t + 5]), W[q][t + 5]));
    if (t + 6 < 64) ZROUND(c, d, e, f, g, h, a, b, ZADD(ZC(kSha256K[t + 6]), W[q][t + 6]));
    if (t + 7 < 64) ZROUND(b, c, d, e, f, g, h, a, ZADD(ZC(kSha256K[t + 7]), W[q][t + 7]));
  }
  // 61 rounds from round 3 leave the variables rotated by 61 mod 8 = 5 places: round t's "a" is in the slot
  // named by (3 - t) mod 8. After round 63 the new a is in slot (3 - 64) mod 8 = 3 -> d, then e..h, a, b, c
  // ---- second hash: the first hash's digest, padding, 256 bits
  __m512i X[G][64];
  __m512i A[G], B[G], Cc[G], D[G], E[G], F[G], Gg[G], H[G];
  for (int q = 0; q < G; ++q) {
    const __m512i o[8] = {d[q], e[q], f[q], g[q], h[q], a[q], b[q], c[q]};
    for (int k = 0; k < 8; ++k) X[q][k] = ZADD(o[k], ZC(mid[k]));
    X[q][8] = ZC(0x80000000u);
    for (int t = 9; t < 15; ++t) X[q][t] = ZC(0);
    X[q][15] = ZC(256);
    A[q] = ZC(kSha256IV[0]); B[q] = ZC(kSha256IV[1]); Cc[q] = ZC(kSha256IV[2]); D[q] = ZC(kSha256IV[3]);
    E[q] = ZC(kSha256IV[4]); F[q] = ZC(kSha256IV[5]); Gg[q] = ZC(kSha256IV[6]); H[q] = ZC(kSha256IV[7]);
  }
  for (int q = 0; q < G; ++q) {  // X16..X31: the terms on the padding words X8..X15 are constants
    __m512i* x = X[q];
    x[16] = ZADD(Zs0(x[1]), x[0]);
    x[17] = ZADD(ZADD(Zs0(x[2]), x[1]), ZC(p.x17));
    for (int t = 18; t < 22; ++t) x[t] = ZADD(ZADD(Zs1(x[t - 2]), Zs0(x[t - 15])), x[t - 16]);
    x[22] = ZADD(ZADD(Zs1(x[20]), Zs0(x[7])), ZADD(x[6], ZC(256)));
    x[23] = ZADD(ZADD(Zs1(x[21]), x[16]), ZADD(x[7], ZC(p.x23)));
    x[24] = ZADD(ZADD(Zs1(x[22]), x[17]), ZC(0x80000000u));
    for (int t = 25; t < 30; ++t) x[t] = ZADD(Zs1(x[t - 2]), x[t - 7]);
    x[30] = ZADD(ZADD(Zs1(x[28]), x[23]), ZC(p.x30));
    x[31] = ZADD(ZADD(Zs1(x[29]), x[24]), ZADD(Zs0(x[16]), ZC(256)));
  }
#pragma GCC unroll 64
  for (int t = 32; t < 61; ++t)
    for (int q = 0; q < G; ++q)
      X[q][t] = ZADD(ZADD(Zs1(X[q][t - 2]), X[q][t - 7]), ZADD(Zs0(X[q][t - 15]), X[q][t - 16]));
  for (int q = 0; q < G; ++q) {  // round 0 on the IV: everything but X0 is constant
    const __m512i t1 = ZADD(ZC(p.r0_t1), X[q][0]);
    D[q] = ZADD(D[q], t1);
    H[q] = ZADD(t1, ZC(p.r0_t2));
  }
#pragma GCC unroll 64
  for (int t = 0; t < 56; t += 8) {
    if (t != 0) ZROUND(A, B, Cc, D, E, F, Gg, H, ZADD(ZC(kSha256K[t]), X[q][t]));
    ZROUND(H, A, B, Cc, D, E, F, Gg, ZADD(ZC(kSha256K[t + 1]), X[q][t + 1]));
    ZROUND(Gg, H, A, B, Cc, D, E, F, ZADD(ZC(kSha256K[t + 2]), X[q][t + 2]));
    ZROUND(F, Gg, H, A, B, Cc, D, E, ZADD(ZC(kSha256K[t + 3]), X[q][t + 3]));
    ZROUND(E, F, Gg, H, A, B, Cc, D, ZADD(ZC(kSha256K[t + 4]), X[q][t + 4]));
    ZROUND(D, E, F, Gg, H, A, B, Cc, ZADD(ZC(kSha256K[t + 5]), X[q][t + 5]));
    ZROUND(Cc, D, E, F, Gg, H, A, B, ZADD(ZC(kSha256K[t + 6]), X[q][t + 6]));
    ZROUND(B, Cc, D, E, F, Gg, H, A, ZADD(ZC(kSha256K[t + 7]), X[q][t + 7]));
  }
  // round 56 in full (its a is d at round 60); rounds 57-59 only their e half (the a values they would make never
  // reach e61); round 60 only as far as e61 = d60 + T1
  ZROUND(A, B, Cc, D, E, F, Gg, H, ZADD(ZC(kSha256K[56]), X[q][56]));
#define ZROUND_E(d, e, f, g, h, kw)                                                 \
  for (int q = 0; q < G; ++q) d[q] = ZADD(d[q], ZADD(ZADD(h[q], ZS1(e[q])), ZADD(ZCH(e[q], f[q], g[q]), (kw))));
  ZROUND_E(Cc, D, E, F, Gg, ZADD(ZC(kSha256K[57]), X[q][57]));
  ZROUND_E(B, Cc, D, E, F, ZADD(ZC(kSha256K[58]), X[q][58]));
  ZROUND_E(A, B, Cc, D, E, ZADD(ZC(kSha256K[59]), X[q][59]));
#undef ZROUND_E
  const __m512i vthi = ZC(thi);
  for (int q = 0; q < G; ++q) {
    // round 60: a = E, b..d = F, G, H, e = A, f..h = B, Cc, D
    const __m512i t1 = ZADD(ZADD(D[q], ZS1(A[q])), ZADD(ZCH(A[q], B[q], Cc[q]), ZADD(ZC(kSha256K[60]), X[q][60])));
    const __m512i h7 = ZADD(ZADD(H[q], t1), ZC(0x5be0cd19u));
    const __mmask16 hit = _mm512_cmple_epu32_mask(_mm512_shuffle_epi8(h7, bswap), vthi);
    if (hit) {
      for (int l = 0; l < 16; ++l)
        if (hit >> l & 1) cands->push_back(n0 + 16u * uint32_t(q) + uint32_t(l));
    }
  }
}

__attribute__((target("avx512f,avx512bw"))) static void sha256d_scan_h7_avx512(int groups, const uint32_t mid[8],
                                                                             const uint8_t tail12[12], uint32_t start,
                                                                             uint64_t count, uint32_t thi,
                                                                             std::vector<uint32_t>* cands,
                                                                             uint64_t* done) {
  // scalar prologue: rounds 0-2 of block 2 and the nonce-free schedule words
  ScanPre p;
  p.w0 = load_be32(tail12); p.w1 = load_be32(tail12 + 4); p.w2 = load_be32(tail12 + 8);
  std::memcpy(p.st, mid, 32);
  auto rotr = [](uint32_t x, int n) { return (x >> n) | (x << (32 - n)); };
  auto round_s = [&](uint32_t* v, uint32_t kw) {
    const uint32_t t1 = v[7] + (rotr(v[4], 6) ^ rotr(v[4], 11) ^ rotr(v[4], 25)) + ((v[4] & v[5]) ^ (~v[4] & v[6])) + kw;
    const uint32_t t2 = (rotr(v[0], 2) ^ rotr(v[0], 13) ^ rotr(v[0], 22)) + ((v[0] & v[1]) ^ (v[0] & v[2]) ^ (v[1] & v[2]));
    for (int i = 7; i > 0; --i) v[i] = v[i - 1];
    v[4] += t1;
    v[0] = t1 + t2;
  };
  round_s(p.st, kSha256K[0] + p.w0);
  round_s(p.st, kSha256K[1] + p.w1);
  round_s(p.st, kSha256K[2] + p.w2);
  auto ss0 = [&](uint32_t x) { return rotr(x, 7) ^ rotr(x, 18) ^ (x >> 3); };
  auto ss1 = [&](uint32_t x) { return rotr(x, 17) ^ rotr(x, 19) ^ (x >> 10); };
  p.w16 = ss1(0) + 0 + ss0(p.w1) + p.w0;    // W14 = 0, W9 = 0
  p.w17 = ss1(640) + 0 + ss0(p.w2) + p.w1;  // W15 = 640, W10 = 0
  p.c18 = ss1(p.w16) + p.w2;                // W18 = c18 + s0(W3)      (W11 = 0)
  p.c19 = ss1(p.w17) + ss0(0x80000000u);    // W19 = c19 + W3          (W12 = 0)
  p.c30 = ss0(640);                         // W30 = s1(W28) + W23 + c30
  p.c31 = ss0(p.w16) + 640;                 // W31 = s1(W29) + W24 + c31
  p.c32 = ss0(p.w17) + p.w16;               // W32 = s1(W30) + W25 + c32
  auto bs1 = [&](uint32_t x) { return rotr(x, 6) ^ rotr(x, 11) ^ rotr(x, 25); };
  auto bs0 = [&](uint32_t x) { return rotr(x, 2) ^ rotr(x, 13) ^ rotr(x, 22); };
  auto ch = [](uint32_t x, uint32_t y, uint32_t z) { return (x & y) ^ (~x & z); };
  auto maj = [](uint32_t x, uint32_t y, uint32_t z) { return (x & y) ^ (x & z) ^ (y & z); };
  p.r3_t1 = p.st[7] + bs1(p.st[4]) + ch(p.st[4], p.st[5], p.st[6]);
  p.r3_t2 = bs0(p.st[0]) + maj(p.st[0], p.st[1], p.st[2]);
  p.x17 = ss1(256);
  p.x23 = ss0(0x80000000u);
  p.x30 = ss0(256);
  p.r0_t1 = kSha256IV[7] + bs1(kSha256IV[4]) + ch(kSha256IV[4], kSha256IV[5], kSha256IV[6]) + kSha256K[0];
  p.r0_t2 = bs0(kSha256IV[0]) + maj(kSha256IV[0], kSha256IV[1], kSha256IV[2]);
  uint64_t i = 0;
  if (groups == 4)
    for (; i + 64 <= count; i += 64) sha256d_h7_x16<4>(p, mid, start + uint32_t(i), thi, cands);
  if (groups == 3)
    for (; i + 48 <= count; i += 48) sha256d_h7_x16<3>(p, mid, start + uint32_t(i), thi, cands);
  if (groups >= 2)
    for (; i + 32 <= count; i += 32) sha256d_h7_x16<2>(p, mid, start + uint32_t(i), thi, cands);
  for (; i + 16 <= count; i += 16) sha256d_h7_x16<1>(p, mid, start + uint32_t(i), thi, cands);
  *done = i;
}
#undef ZROUND
#undef ZADD
#undef ZC
#undef ZMAJ
#undef ZCH
#undef Zs1
#undef Zs0
#undef ZS1
#undef ZS0
#undef ZROR

bool cpu_has_avx512_sha_scan() {
  static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
  return ok;
}

int sha256d_scan_wide_groups() {
  static const int groups = [] {
    const char* v = std::getenv("OTEDAMA_CPU_SCAN_GROUPS");  // A/B: 16-lane groups in flight per step (1..4)
    const int n = v ? std::atoi(v) : 0;
    if (n >= 1 && n <= 4) return n;
    // Measured single thread (tools/cpu_scan_ab.py, profiles/r4/r_cpu_avx512): AMD EPYC 9575F (Zen 5) 41.4 / 51.3 /
    // 46.8 / 38.7 MH/s for 1-4 groups; the build container's Intel Xeon 28.1 / 24.4 / 21.9 / 19.2 (its 32 zmm
    // registers spill from two groups on, where Zen 5's renamer and store forwarding absorb the spills).
    unsigned a = 0, b = 0, c = 0, d = 0;
    char vendor[13] = {0};
    if (__get_cpuid(0, &a, &b, &c, &d)) {
      std::memcpy(vendor, &b, 4);
      std::memcpy(vendor + 4, &d, 4);
      std::memcpy(vendor + 8, &c, 4);
    }
    return std::strcmp(vendor, "AuthenticAMD") == 0 ? 2 : 1;
  }();
  return groups;
}

bool sha256d_scan_h7_wide(const uint32_t mid[8], const uint8_t tail12[12], uint32_t start, uint64_t count,
                          uint32_t thi, std::vector<uint32_t>* cands, uint64_t* done) {
  if (!cpu_has_avx512_sha_scan()) return false;
  sha256d_scan_h7_avx512(sha256d_scan_wide_groups(), mid, tail12, start, count, thi, cands, done);
  return true;
}

bool sha256d_scan_h7(int lanes, const uint32_t mid[8], const uint8_t tail12[12], uint32_t start, uint64_t count,
                     uint32_t thi, std::vector<uint32_t>* cands, uint64_t* done) {
  if (!cpu_has_sha_ni()) return false;
  sha256d_scan_h7_shani(lanes, mid, tail12, start, count, thi, cands, done);
  return true;
}

static bool detect_sha_ni() {
  unsigned a, b, c, d;
  bool ok = false;
  if (__get_cpuid_count(7, 0, &a, &b, &c, &d)) ok = (b >> 29) & 1;  // EBX bit 29 = SHA
  unsigned a1, b1, c1, d1;
  if (ok && __get_cpuid(1, &a1, &b1, &c1, &d1)) ok = (c1 >> 19) & 1;  // SSE4.1
  return ok;
}

bool cpu_has_sha_ni() {
  // Function-local static: thread-safe one-time init (a plain lazily-written int raced
  // across miner threads; found by tools/sanitize under TSan).
  static const bool cached = detect_sha_ni();
  return cached;
}

void sha256_compress(uint32_t state[8], const uint8_t block[64]) {
  if (cpu_has_sha_ni()) sha256_compress_shani(state, block);
  else sha256_compress_portable(state, block);
}

void sha256_compress_x2(uint32_t s0[8], const uint8_t b0[64], uint32_t s1[8], const uint8_t b1[64]) {
  if (cpu_has_sha_ni()) {
    uint32_t* const st[2] = {s0, s1};
    const uint8_t* const bl[2] = {b0, b1};
    sha256_compress_shani_xn<2>(st, bl);
  } else {
    sha256_compress_portable(s0, b0);
    sha256_compress_portable(s1, b1);
  }
}

void sha256_compress_xn(int n, uint32_t* const state[], const uint8_t* const block[]) {
  if (!cpu_has_sha_ni()) {
    for (int i = 0; i < n; ++i) sha256_compress_portable(state[i], block[i]);
    return;
  }
  int i = 0;
  for (; i + 4 <= n; i += 4) sha256_compress_shani_xn<4>(state + i, block + i);
  if (n - i == 3) sha256_compress_shani_xn<3>(state + i, block + i);
  else if (n - i == 2) sha256_compress_shani_xn<2>(state + i, block + i);
  else if (n - i == 1) sha256_compress_shani(state[i], block[i]);
}

void sha256(const uint8_t* data, size_t len, uint8_t out[32]) {
  uint32_t st[8];
  std::memcpy(st, kSha256IV, sizeof st);
  size_t off = 0;
  while (len - off >= 64) { sha256_compress(st, data + off); off += 64; }
  uint8_t tail[128] = {0};
  size_t rem = len - off;
  if (rem) std::memcpy(tail, data + off, rem);  // data may be null when len == 0
  tail[rem] = 0x80;
  size_t tl = (rem + 9 <= 64) ? 64 : 128;
  uint64_t bits = uint64_t(len) * 8;
  for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = uint8_t(bits >> (8 * i));
  sha256_compress(st, tail);
  if (tl == 128) sha256_compress(st, tail + 64);
  for (int i = 0; i < 8; ++i) store_be32(out + 4 * i, st[i]);
}

void sha256d(const uint8_t* data, size_t len, uint8_t out[32]) {
  uint8_t h[32];
  sha256(data, len, h);
  sha256(h, 32, out);
}

void hmac_sha256(const uint8_t* key, size_t klen, const uint8_t* msg, size_t mlen, uint8_t out[32]) {
  uint8_t k[64] = {0};
  if (klen > 64) sha256(key, klen, k);
  else if (klen) std::memcpy(k, key, klen);  // key may be null when klen == 0
  uint8_t ipad[64], opad[64];
  for (int i = 0; i < 64; ++i) { ipad[i] = k[i] ^ 0x36; opad[i] = k[i] ^ 0x5c; }
  // inner = H(ipad || msg)
  uint32_t st[8];
  std::memcpy(st, kSha256IV, sizeof st);
  sha256_compress(st, ipad);
  size_t off = 0;
  while (mlen - off >= 64) { sha256_compress(st, msg + off); off += 64; }
  uint8_t tail[128] = {0};
  size_t rem = mlen - off;
  if (rem) std::memcpy(tail, msg + off, rem);
  tail[rem] = 0x80;
  size_t tl = (rem + 9 <= 64) ? 64 : 128;
  uint64_t bits = uint64_t(64 + mlen) * 8;
  for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = uint8_t(bits >> (8 * i));
  sha256_compress(st, tail);
  if (tl == 128) sha256_compress(st, tail + 64);
  uint8_t inner[32];
  for (int i = 0; i < 8; ++i) store_be32(inner + 4 * i, st[i]);
  // outer = H(opad || inner)
  std::memcpy(st, kSha256IV, sizeof st);
  sha256_compress(st, opad);
  uint8_t blk[64] = {0};
  std::memcpy(blk, inner, 32);
  blk[32] = 0x80;
  blk[62] = 0x03;  // (64 + 32) * 8 = 768 = 0x300
  blk[63] = 0x00;
  sha256_compress(st, blk);
  for (int i = 0; i < 8; ++i) store_be32(out + 4 * i, st[i]);
}

void pbkdf2_sha256(const uint8_t* pw, size_t pwlen, const uint8_t* salt, size_t saltlen,
                   uint32_t iters, uint8_t* out, size_t outlen) {
  uint8_t buf[1024];
  uint8_t* msg = saltlen + 4 <= sizeof buf ? buf : new uint8_t[saltlen + 4];
  if (saltlen) std::memcpy(msg, salt, saltlen);
  uint32_t blockno = 1;
  size_t done = 0;
  while (done < outlen) {
    msg[saltlen] = uint8_t(blockno >> 24); msg[saltlen + 1] = uint8_t(blockno >> 16);
    msg[saltlen + 2] = uint8_t(blockno >> 8); msg[saltlen + 3] = uint8_t(blockno);
    uint8_t u[32], t[32];
    hmac_sha256(pw, pwlen, msg, saltlen + 4, u);
    std::memcpy(t, u, 32);
    for (uint32_t it = 1; it < iters; ++it) {
      hmac_sha256(pw, pwlen, u, 32, u);
      for (int j = 0; j < 32; ++j) t[j] ^= u[j];
    }
    size_t n = outlen - done < 32 ? outlen - done : 32;
    std::memcpy(out + done, t, n);
    done += n;
    ++blockno;
  }
  if (msg != buf) delete[] msg;
}

}  // namespace otedama
