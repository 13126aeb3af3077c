// Host-side per-job folding for the gfx950 search kernels (see job.h).
#include "otedama/job.h"
#include "otedama/sha256.h"

namespace otedama {

static inline uint32_t S0(uint32_t a) { return rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22); }
static inline uint32_t S1(uint32_t e) { return rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25); }
static inline uint32_t s0(uint32_t x) { return rotr32(x, 7) ^ rotr32(x, 18) ^ (x >> 3); }
static inline uint32_t s1(uint32_t x) { return rotr32(x, 17) ^ rotr32(x, 19) ^ (x >> 10); }
static inline uint32_t Ch(uint32_t e, uint32_t f, uint32_t g) { return (e & f) ^ (~e & g); }
static inline uint32_t Maj(uint32_t a, uint32_t b, uint32_t c) { return (a & b) ^ (a & c) ^ (b & c); }

void sha256d_prepare(const uint8_t header80[80], const uint8_t target32[32], Sha256dParams* p) {
  uint32_t st[8];
  for (int i = 0; i < 8; ++i) st[i] = kSha256IV[i];
  sha256_compress_portable(st, header80);
  for (int i = 0; i < 8; ++i) p->mid[i] = st[i];
  uint32_t W[16] = {0};
  W[0] = load_be32(header80 + 64);
  W[1] = load_be32(header80 + 68);
  W[2] = load_be32(header80 + 72);
  W[4] = 0x80000000u;
  W[15] = 640u;
  p->w0 = W[0]; p->w1 = W[1]; p->w2 = W[2];
  // W16 = s1(W14) + W9 + s0(W1) + W0 ; W17 = s1(W15) + W10 + s0(W2) + W1
  p->w16 = s1(W[14]) + W[9] + s0(W[1]) + W[0];
  p->w17 = s1(W[15]) + W[10] + s0(W[2]) + W[1];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int t = 0; t < 3; ++t) {
    uint32_t t1 = h + S1(e) + Ch(e, f, g) + kSha256K[t] + W[t];
    uint32_t t2 = S0(a) + Maj(a, b, c);
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  p->st3[0] = a; p->st3[1] = b; p->st3[2] = c; p->st3[3] = d;
  p->st3[4] = e; p->st3[5] = f; p->st3[6] = g; p->st3[7] = h;
  p->pre3 = h + S1(e) + Ch(e, f, g) + kSha256K[3];
  p->t2_3 = S0(a) + Maj(a, b, c);
  p->target_hi = load_le32(target32 + 28);
}

void scrypt_prepare(const uint8_t header80[80], const uint8_t target32[32], ScryptParams* p) {
  for (int i = 0; i < 19; ++i) p->hdr[i] = load_le32(header80 + 4 * i);
  uint32_t st[8];
  for (int i = 0; i < 8; ++i) st[i] = kSha256IV[i];
  sha256_compress_portable(st, header80);
  for (int i = 0; i < 8; ++i) p->hmid[i] = st[i];
  p->target_hi = load_le32(target32 + 28);
}

}  // namespace otedama

namespace otedama {

bool sha256d_prepare_k(const uint8_t* const headers80[], int k, const uint8_t target32[32], Sha256dParamsK* out) {
  if (k < 2 || k > kSha256dMaxK || sha256d_k_floor(k) != k) return false;
  for (int v = 1; v < k; ++v)
    for (int i = 64; i < 76; ++i)
      if (headers80[v][i] != headers80[0][i]) return false;
  for (int v = 0; v < k; ++v) {
    Sha256dParams p;
    sha256d_prepare(headers80[v], target32, &p);
    if (v == 0) {
      out->w0 = p.w0; out->w1 = p.w1; out->w2 = p.w2; out->w16 = p.w16; out->w17 = p.w17;
      out->target_hi = p.target_hi;
    }
    for (int i = 0; i < 8; ++i) { out->var[v].mid[i] = p.mid[i]; out->var[v].st3[i] = p.st3[i]; }
    out->var[v].pre3 = p.pre3;
    out->var[v].t2_3 = p.t2_3;
  }
  for (int v = k; v < kSha256dMaxK; ++v) out->var[v] = out->var[0];
  out->k = k;
  return true;
}

bool sha256d_prepare_v(const uint8_t* const headers80[], int n, const uint8_t target32[32], Sha256dParamsV* p,
                       Sha256dVariant* vars) {
  if (n <= 0 || n % kSha256dVGroup != 0) return false;
  for (int v = 1; v < n; ++v)
    for (int i = 64; i < 76; ++i)
      if (headers80[v][i] != headers80[0][i]) return false;
  for (int v = 0; v < n; ++v) {
    Sha256dParams q;
    sha256d_prepare(headers80[v], target32, &q);
    if (v == 0) {
      p->w0 = q.w0; p->w1 = q.w1; p->w2 = q.w2; p->w16 = q.w16; p->w17 = q.w17;
      p->target_hi = q.target_hi;
    }
    for (int i = 0; i < 8; ++i) { vars[v].mid[i] = q.mid[i]; vars[v].st3[i] = q.st3[i]; }
    vars[v].pre3 = q.pre3;
    vars[v].t2_3 = q.t2_3;
  }
  p->groups = uint32_t(n / kSha256dVGroup);
  p->occupancy8 = 0;
  return true;
}

void x11_prepare(const uint8_t header80[80], const uint8_t target32[32], X11Params* p) {
  for (int k = 0; k < 9; ++k) p->m[k] = (uint64_t(load_be32(header80 + 8 * k)) << 32) | load_be32(header80 + 8 * k + 4);
  p->m9_hi = uint64_t(load_be32(header80 + 72)) << 32;
  p->target_hi = (uint64_t(load_le32(target32 + 28)) << 32) | load_le32(target32 + 24);
}

}  // namespace otedama
