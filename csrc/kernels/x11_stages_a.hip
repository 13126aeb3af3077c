// X11 stages 1-8 on gfx950: BLAKE-512 (80-byte header), BMW-512, Groestl-512,
// Skein-512, JH-512, Keccak-512, Luffa-512, CubeHash16/32-512 (64-byte inputs). One lane per nonce; the padding
// blocks of the fixed-length inputs are folded into compile-time constants.
// Bit-exact oracle: csrc/cpu/x11_cpu.cpp (tests/test_x11_gpu.py compares every stage).
#include "x11_common.h"

namespace otedama {
namespace x11k {

// ------------------------------------------------------------------ BLAKE-512
constexpr u64 kBlakeC[16] = {
    0x243F6A8885A308D3ull, 0x13198A2E03707344ull, 0xA4093822299F31D0ull, 0x082EFA98EC4E6C89ull,
    0x452821E638D01377ull, 0xBE5466CF34E90C6Cull, 0xC0AC29B7C97C50DDull, 0x3F84D5B5B5470917ull,
    0x9216D5D98979FB1Bull, 0xD1310BA698DFB5ACull, 0x2FFD72DBD01ADFB7ull, 0xB8E1AFED6A267E96ull,
    0xBA7C9045F12C7F99ull, 0x24A19947B3916CF7ull, 0x0801F2E2858EFC16ull, 0x636920D871574E69ull};
constexpr unsigned char kSigma[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};
constexpr u64 kSha512Iv[8] = {0x6A09E667F3BCC908ull, 0xBB67AE8584CAA73Bull, 0x3C6EF372FE94F82Bull, 0xA54FF53A5F1D36F1ull,
                              0x510E527FADE682D1ull, 0x9B05688C2B3E6C1Full, 0x1F83D9ABFB41BD6Bull, 0x5BE0CD19137E2179ull};

#define BLAKE_G(a, b, c, d, x, y)                 \
  do {                                            \
    v[a] = v[a] + v[b] + (m[x] ^ kBlakeC[y]);     \
    v[d] = rotr64(v[d] ^ v[a], 32);               \
    v[c] = v[c] + v[d];                           \
    v[b] = rotr64(v[b] ^ v[c], 25);               \
    v[a] = v[a] + v[b] + (m[y] ^ kBlakeC[x]);     \
    v[d] = rotr64(v[d] ^ v[a], 16);               \
    v[c] = v[c] + v[d];                           \
    v[b] = rotr64(v[b] ^ v[c], 11);               \
  } while (0)

__device__ __forceinline__ void blake512_80(const X11Params& p, u32 nonce, u64 h[8]) {
  u64 m[16];
#pragma unroll
  for (int k = 0; k < 9; ++k) m[k] = p.m[k];
  m[9] = p.m9_hi | bswap32(nonce);
  m[10] = 0x8000000000000000ull;
  m[11] = 0; m[12] = 0; m[13] = 1; m[14] = 0; m[15] = 640;
  u64 v[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = kSha512Iv[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[8 + k] = kBlakeC[k];
  v[12] = 640 ^ kBlakeC[4];
  v[13] = 640 ^ kBlakeC[5];
  v[14] = kBlakeC[6];
  v[15] = kBlakeC[7];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const unsigned char* s = kSigma[r % 10];
    BLAKE_G(0, 4, 8, 12, s[0], s[1]);
    BLAKE_G(1, 5, 9, 13, s[2], s[3]);
    BLAKE_G(2, 6, 10, 14, s[4], s[5]);
    BLAKE_G(3, 7, 11, 15, s[6], s[7]);
    BLAKE_G(0, 5, 10, 15, s[8], s[9]);
    BLAKE_G(1, 6, 11, 12, s[10], s[11]);
    BLAKE_G(2, 7, 8, 13, s[12], s[13]);
    BLAKE_G(3, 4, 9, 14, s[14], s[15]);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = bswap64(kSha512Iv[k] ^ v[k] ^ v[k + 8]);
}
#undef BLAKE_G

// ------------------------------------------------------------------ BMW-512
__device__ __forceinline__ u64 bs0(u64 x) { return (x >> 1) ^ (x << 3) ^ rotl64(x, 4) ^ rotl64(x, 37); }
__device__ __forceinline__ u64 bs1(u64 x) { return (x >> 1) ^ (x << 2) ^ rotl64(x, 13) ^ rotl64(x, 43); }
__device__ __forceinline__ u64 bs2(u64 x) { return (x >> 2) ^ (x << 1) ^ rotl64(x, 19) ^ rotl64(x, 53); }
__device__ __forceinline__ u64 bs3(u64 x) { return (x >> 2) ^ (x << 2) ^ rotl64(x, 28) ^ rotl64(x, 59); }
__device__ __forceinline__ u64 bs4(u64 x) { return (x >> 1) ^ x; }
__device__ __forceinline__ u64 bs5(u64 x) { return (x >> 2) ^ x; }

__device__ __forceinline__ void bmw_compress(u64 H[16], const u64 M[16]) {
  u64 X[16], Q[32];
#pragma unroll
  for (int k = 0; k < 16; ++k) X[k] = M[k] ^ H[k];
  Q[0] = bs0(X[5] - X[7] + X[10] + X[13] + X[14]) + H[1];
  Q[1] = bs1(X[6] - X[8] + X[11] + X[14] - X[15]) + H[2];
  Q[2] = bs2(X[0] + X[7] + X[9] - X[12] + X[15]) + H[3];
  Q[3] = bs3(X[0] - X[1] + X[8] - X[10] + X[13]) + H[4];
  Q[4] = bs4(X[1] + X[2] + X[9] - X[11] - X[14]) + H[5];
  Q[5] = bs0(X[3] - X[2] + X[10] - X[12] + X[15]) + H[6];
  Q[6] = bs1(X[4] - X[0] - X[3] - X[11] + X[13]) + H[7];
  Q[7] = bs2(X[1] - X[4] - X[5] - X[12] - X[14]) + H[8];
  Q[8] = bs3(X[2] - X[5] - X[6] + X[13] - X[15]) + H[9];
  Q[9] = bs4(X[0] - X[3] + X[6] - X[7] + X[14]) + H[10];
  Q[10] = bs0(X[8] - X[1] - X[4] - X[7] + X[15]) + H[11];
  Q[11] = bs1(X[8] - X[0] - X[2] - X[5] + X[9]) + H[12];
  Q[12] = bs2(X[1] + X[3] - X[6] - X[9] + X[10]) + H[13];
  Q[13] = bs3(X[2] + X[4] + X[7] + X[10] + X[11]) + H[14];
  Q[14] = bs4(X[3] - X[5] + X[8] - X[11] - X[12]) + H[15];
  Q[15] = bs0(X[12] - X[4] - X[6] - X[9] + X[13]) + H[0];
#pragma unroll
  for (int j = 16; j < 32; ++j) {
    const int jj = j - 16;
    u64 add = rotl64(M[jj & 15], (jj & 15) + 1) + rotl64(M[(jj + 3) & 15], ((jj + 3) & 15) + 1) -
              rotl64(M[(jj + 10) & 15], ((jj + 10) & 15) + 1) + (u64)j * 0x0555555555555555ull;
    add ^= H[(jj + 7) & 15];
    u64 q;
    if (j < 18) {
      q = bs1(Q[j - 16]) + bs2(Q[j - 15]) + bs3(Q[j - 14]) + bs0(Q[j - 13]) + bs1(Q[j - 12]) + bs2(Q[j - 11]) +
          bs3(Q[j - 10]) + bs0(Q[j - 9]) + bs1(Q[j - 8]) + bs2(Q[j - 7]) + bs3(Q[j - 6]) + bs0(Q[j - 5]) +
          bs1(Q[j - 4]) + bs2(Q[j - 3]) + bs3(Q[j - 2]) + bs0(Q[j - 1]);
    } else {
      q = Q[j - 16] + rotl64(Q[j - 15], 5) + Q[j - 14] + rotl64(Q[j - 13], 11) + Q[j - 12] + rotl64(Q[j - 11], 27) +
          Q[j - 10] + rotl64(Q[j - 9], 32) + Q[j - 8] + rotl64(Q[j - 7], 37) + Q[j - 6] + rotl64(Q[j - 5], 43) +
          Q[j - 4] + rotl64(Q[j - 3], 53) + bs4(Q[j - 2]) + bs5(Q[j - 1]);
    }
    Q[j] = q + add;
  }
  u64 XL = Q[16] ^ Q[17] ^ Q[18] ^ Q[19] ^ Q[20] ^ Q[21] ^ Q[22] ^ Q[23];
  u64 XH = XL ^ Q[24] ^ Q[25] ^ Q[26] ^ Q[27] ^ Q[28] ^ Q[29] ^ Q[30] ^ Q[31];
  H[0] = ((XH << 5) ^ (Q[16] >> 5) ^ M[0]) + (XL ^ Q[24] ^ Q[0]);
  H[1] = ((XH >> 7) ^ (Q[17] << 8) ^ M[1]) + (XL ^ Q[25] ^ Q[1]);
  H[2] = ((XH >> 5) ^ (Q[18] << 5) ^ M[2]) + (XL ^ Q[26] ^ Q[2]);
  H[3] = ((XH >> 1) ^ (Q[19] << 5) ^ M[3]) + (XL ^ Q[27] ^ Q[3]);
  H[4] = ((XH >> 3) ^ Q[20] ^ M[4]) + (XL ^ Q[28] ^ Q[4]);
  H[5] = ((XH << 6) ^ (Q[21] >> 6) ^ M[5]) + (XL ^ Q[29] ^ Q[5]);
  H[6] = ((XH >> 4) ^ (Q[22] << 6) ^ M[6]) + (XL ^ Q[30] ^ Q[6]);
  H[7] = ((XH >> 11) ^ (Q[23] << 2) ^ M[7]) + (XL ^ Q[31] ^ Q[7]);
  H[8] = rotl64(H[4], 9) + (XH ^ Q[24] ^ M[8]) + ((XL << 8) ^ Q[23] ^ Q[8]);
  H[9] = rotl64(H[5], 10) + (XH ^ Q[25] ^ M[9]) + ((XL >> 6) ^ Q[16] ^ Q[9]);
  H[10] = rotl64(H[6], 11) + (XH ^ Q[26] ^ M[10]) + ((XL << 6) ^ Q[17] ^ Q[10]);
  H[11] = rotl64(H[7], 12) + (XH ^ Q[27] ^ M[11]) + ((XL << 4) ^ Q[18] ^ Q[11]);
  H[12] = rotl64(H[0], 13) + (XH ^ Q[28] ^ M[12]) + ((XL >> 3) ^ Q[19] ^ Q[12]);
  H[13] = rotl64(H[1], 14) + (XH ^ Q[29] ^ M[13]) + ((XL >> 4) ^ Q[20] ^ Q[13]);
  H[14] = rotl64(H[2], 15) + (XH ^ Q[30] ^ M[14]) + ((XL >> 7) ^ Q[21] ^ Q[14]);
  H[15] = rotl64(H[3], 16) + (XH ^ Q[31] ^ M[15]) + ((XL >> 2) ^ Q[22] ^ Q[15]);
}

__device__ __forceinline__ void bmw512_64(u64 h[8]) {
  u64 M[16], H[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) M[k] = h[k];
  M[8] = 0x80; M[9] = 0; M[10] = 0; M[11] = 0; M[12] = 0; M[13] = 0; M[14] = 0; M[15] = 512;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const u64 b = 0x80 + 8 * k;
    H[k] = (b << 56) | ((b + 1) << 48) | ((b + 2) << 40) | ((b + 3) << 32) | ((b + 4) << 24) | ((b + 5) << 16) |
           ((b + 6) << 8) | (b + 7);
  }
  bmw_compress(H, M);
  u64 F[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) F[k] = 0xAAAAAAAAAAAAAAA0ull + (u64)k;
  bmw_compress(F, H);
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = F[8 + k];
}

// ------------------------------------------------------------------ Groestl-512
// Column j of the 8x16 byte state is one 64-bit word (row r in byte r). Output column j is
// XOR_r T_r[row r byte of column (j + shift_r) mod 16] with T_r = rotl64(T0, 8r). Rows r and r+4
// differ by a half swap (free), so with L_r = T0[b_r] ^ swap(T0[b_(r+4)]) the column is
// L0 ^ rotl8(L1 ^ rotl8(L2 ^ rotl8(L3))): 8 conflict-free lookups from the lane's private T0
// copy, 3 64-bit rotates, 4 64-bit (x)xor3s.
constexpr int kGroestlBlock = 512;
__device__ __forceinline__ u64 swap64(u64 x) { return mk64(hi32(x), lo32(x)); }

template <bool kQ>
__device__ __forceinline__ void groestl_arc(u64 a[16], u32 r) {  // AddRoundConstant
  if (!kQ) {
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] ^= (u64)(((u32)j << 4) ^ r);
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = mk64(~lo32(a[j]), hi32(a[j]) ^ ~((((u32)j << 4) ^ r) << 24));
  }
}

// Output column j of one round (SubBytes + ShiftBytes + MixBytes). Columns >= kConstFrom of `a` are compile-time
// constants (round 0 of a one-block message: the padding half), so their lookups come from the constant table and
// fold away instead of reading LDS.
template <bool kQ, int kConstFrom>
__device__ __forceinline__ u64 groestl_col(const u64* T, u32 lo, const u64 a[16], int j) {
  constexpr int SP[8] = {0, 1, 2, 3, 4, 5, 6, 11};
  constexpr int SQ[8] = {1, 3, 5, 11, 0, 2, 4, 6};
  u64 v[8];
#pragma unroll
  for (int row = 0; row < 8; ++row) {
    const int col = (j + (kQ ? SQ[row] : SP[row])) & 15;
    const u32 w = row < 4 ? lo32(a[col]) : hi32(a[col]);
    v[row] = col >= kConstFrom ? x11t::GROESTL_T0[(w >> (8 * (row & 3))) & 0xFF] : groestl_lk(T, lo, w, row & 3);
  }
  const u64 L3 = v[3] ^ swap64(v[7]);
  const u64 L2 = xor3_64(v[2], swap64(v[6]), rotl64(L3, 8));
  const u64 L1 = xor3_64(v[1], swap64(v[5]), rotl64(L2, 8));
  return xor3_64(v[0], swap64(v[4]), rotl64(L1, 8));
}

// kConstFrom: first compile-time-constant column of the input (16: none). kHalfOut: only columns 8..15 of the
// result are used (the output transform), so the last round computes just those.
template <bool kQ, int kConstFrom = 16, bool kHalfOut = false>
__device__ __forceinline__ void groestl_perm(const u64* T, u32 lo, u64 a[16]) {
  u64 t[16];
  groestl_arc<kQ>(a, 0);
#pragma unroll
  for (int j = 0; j < 16; ++j) t[j] = groestl_col<kQ, kConstFrom>(T, lo, a, j);
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = t[j];
#pragma unroll 1
  for (u32 r = 1; r < (kHalfOut ? 13u : 14u); ++r) {
    groestl_arc<kQ>(a, r);
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = groestl_col<kQ, 16>(T, lo, a, j);
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = t[j];
  }
  if (kHalfOut) {
    groestl_arc<kQ>(a, 13);
#pragma unroll
    for (int j = 8; j < 16; ++j) t[j] = groestl_col<kQ, 16>(T, lo, a, j);
#pragma unroll
    for (int j = 8; j < 16; ++j) a[j] = t[j];
  }
}

__global__ __launch_bounds__(kGroestlBlock) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_groestl512_64(
    u64* __restrict__ Hb, u32 stride, u32 n, X11Abort ab) {
  __shared__ u64 T[kGroestlPrivQwords];
  groestl_priv_fill(T);
  const u32 lo = groestl_laneoff();
  for (u32 i = blockIdx.x * kGroestlBlock + threadIdx.x; i < n; i += gridDim.x * kGroestlBlock) {
    u64 m[16], p[16], q[16];
    const u32 a0 = x11_abort_issue(ab);
    load_hash(Hb, stride, i, m);
    if (x11_abort_seen(a0, ab)) return;
    m[8] = 0x80;
#pragma unroll
    for (int k = 9; k < 15; ++k) m[k] = 0;
    m[15] = 0x0100000000000000ull;  // one block, 64-bit big-endian count
    const u64 iv15 = 0x0002000000000000ull;  // 512 in the last bytes of h
#pragma unroll
    for (int k = 0; k < 16; ++k) { p[k] = m[k]; q[k] = m[k]; }
    p[15] ^= iv15;
    groestl_perm<false, 8>(T, lo, p);  // columns 8..15 (padding, and h's length word) are constants
    groestl_perm<true, 8>(T, lo, q);
#pragma unroll
    for (int k = 0; k < 16; ++k) p[k] ^= q[k];
    p[15] ^= iv15;  // h' = P(h^m) ^ Q(m) ^ h
#pragma unroll
    for (int k = 0; k < 16; ++k) q[k] = p[k];
    groestl_perm<false, 16, true>(T, lo, q);  // output transform: only columns 8..15 are kept
    u64 out[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = q[8 + k] ^ p[8 + k];
    store_hash(Hb, stride, i, out);
  }
}

// ------------------------------------------------------------------ Skein-512
constexpr int kSkeinR[8][4] = {{46, 36, 19, 37}, {33, 27, 14, 42}, {17, 49, 36, 39}, {44, 9, 54, 56},
                               {39, 30, 34, 24}, {13, 50, 10, 17}, {25, 29, 39, 43}, {8, 35, 56, 22}};

__device__ __forceinline__ void threefish512(const u64 key[8], u64 t0, u64 t1, u64 v[8]) {
  u64 k[9];
  k[8] = 0x1BD11BDAA9FC1A22ull;
#pragma unroll
  for (int j = 0; j < 8; ++j) { k[j] = key[j]; k[8] ^= key[j]; }
  const u64 t[3] = {t0, t1, t0 ^ t1};
#pragma unroll
  for (int d = 0; d < 72; ++d) {
    if ((d & 3) == 0) {
      const int s = d / 4;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += k[(s + j) % 9];
      v[5] += t[s % 3];
      v[6] += t[(s + 1) % 3];
      v[7] += (u64)s;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] += v[2 * j + 1];
      v[2 * j + 1] = rotl64(v[2 * j + 1], kSkeinR[d & 7][j]) ^ v[2 * j];
    }
    const u64 p0 = v[2], p1 = v[1], p2 = v[4], p3 = v[7], p4 = v[6], p5 = v[5], p6 = v[0], p7 = v[3];
    v[0] = p0; v[1] = p1; v[2] = p2; v[3] = p3; v[4] = p4; v[5] = p5; v[6] = p6; v[7] = p7;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] += k[(18 + j) % 9];
  v[5] += t[0];
  v[6] += t[1];
  v[7] += 18;
}

__device__ __forceinline__ void skein512_64(u64 io[8]) {
  u64 m[8], v[8], h[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { m[k] = io[k]; v[k] = m[k]; h[k] = x11t::SKEIN_IV[k]; }
  threefish512(h, 64, 0xF000000000000000ull, v);  // message: first|final, type 48, position 64
#pragma unroll
  for (int k = 0; k < 8; ++k) { h[k] = v[k] ^ m[k]; v[k] = 0; }
  threefish512(h, 8, 0xFF00000000000000ull, v);   // output: first|final, type 63, position 8
#pragma unroll
  for (int k = 0; k < 8; ++k) io[k] = v[k];
}

// ------------------------------------------------------------------ JH-512
// Bitsliced E8 on the state kept in memory order (x[k][w] = LE u32 word w of
// bytes 16k..16k+15); constants re-labelled from the spec constants by
// tools/gen_x11_tables.cpp, which checks this formulation against the spec form.

// The JH authors' bitsliced S-box layer (constant bit cc selects S0/S1) with every and/or/not + xor
// pair as one v_bitop3 (truth tables for a = 0xF0, b = 0xCC, c = 0xAA); the complement of m3 is
// folded into its three uses. 10 VALU per 4 planes (hipcc alone: ~20).
#define JH_SB4(m0, m1, m2, m3, cc)                 \
  do {                                              \
    u32 t_;                                         \
    m0 = bop3<0xD2>(m0, m2, cc);   /* m0 ^= ~m2 & cc */        \
    t_ = bop3<0x78>(cc, m0, m1);   /* t = cc ^ (m0 & m1) */    \
    m0 = bop3<0xB4>(m0, m2, m3);   /* m0 ^= m2 & ~M3 */        \
    m3 = bop3<0x2D>(m3, m1, m2);   /* m3 = ~M3 ^ (~m1 & m2) */ \
    m1 = bop3<0x78>(m1, m0, m2);   /* m1 ^= m0 & m2 */         \
    m2 = bop3<0xB4>(m2, m0, m3);   /* m2 ^= m0 & ~m3 */        \
    m0 = bop3<0x1E>(m0, m1, m3);   /* m0 ^= m1 | m3 */         \
    m3 = bop3<0x78>(m3, m1, m2);   /* m3 ^= m1 & m2 */         \
    m1 = bop3<0x78>(m1, t_, m0);   /* m1 ^= t & m0 */          \
    m2 ^= t_;                                       \
  } while (0)
#define JH_SS(m0, m1, m2, m3, m4, m5, m6, m7, cc0, cc1) \
  do {                                                  \
    JH_SB4(m0, m1, m2, m3, cc0);                        \
    JH_SB4(m4, m5, m6, m7, cc1);                        \
  } while (0)
#define JH_L(m0, m1, m2, m3, m4, m5, m6, m7) \
  do {                                       \
    m4 ^= m1; m5 ^= m2; m6 = xor3(m6, m0, m3); m7 ^= m0; \
    m0 ^= m5; m1 ^= m6; m2 = xor3(m2, m4, m7); m3 ^= m4; \
  } while (0)

template <int K>
__device__ __forceinline__ u32 jh_swap(u32 x) {
  if (K == 0) return ((x & 0x55555555u) << 1) | ((x >> 1) & 0x55555555u);
  if (K == 1) return ((x & 0x33333333u) << 2) | ((x >> 2) & 0x33333333u);
  if (K == 2) return ((x & 0x0F0F0F0Fu) << 4) | ((x >> 4) & 0x0F0F0F0Fu);
  if (K == 3) return __builtin_amdgcn_perm(x, x, 0x02030001u);  // swap bytes within each 16-bit half
  return rotl32(x, 16);
}

template <int K>
__device__ __forceinline__ void jh_round(u32 x[8][4], const u32* c) {
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    JH_SS(x[0][w], x[2][w], x[4][w], x[6][w], x[1][w], x[3][w], x[5][w], x[7][w], c[w], c[4 + w]);
    JH_L(x[0][w], x[2][w], x[4][w], x[6][w], x[1][w], x[3][w], x[5][w], x[7][w]);
  }
#pragma unroll
  for (int o = 1; o < 8; o += 2) {
    if (K < 5) {
#pragma unroll
      for (int w = 0; w < 4; ++w) x[o][w] = jh_swap<K>(x[o][w]);
    } else if (K == 5) {
      u32 t = x[o][0]; x[o][0] = x[o][1]; x[o][1] = t;
      t = x[o][2]; x[o][2] = x[o][3]; x[o][3] = t;
    } else {
      u32 t = x[o][0]; x[o][0] = x[o][2]; x[o][2] = t;
      t = x[o][1]; x[o][1] = x[o][3]; x[o][3] = t;
    }
  }
}

// BC: the 42 x 8 round constants (x11t::JH_BC, or an LDS copy in the variants of tools/x11_variants.hip). An SGPR
// operand would put v_bitop3 in the slow issue class (profiles/r1/x11/NOTES.md), so each word is moved to a VGPR.
__device__ __forceinline__ void jh_E8(u32 x[8][4], const u32 (*BC)[8]) {
  for (int r = 0; r < 42; r += 7) {
    jh_round<0>(x, BC[r + 0]);
    jh_round<1>(x, BC[r + 1]);
    jh_round<2>(x, BC[r + 2]);
    jh_round<3>(x, BC[r + 3]);
    jh_round<4>(x, BC[r + 4]);
    jh_round<5>(x, BC[r + 5]);
    jh_round<6>(x, BC[r + 6]);
  }
}

// kReload: re-read the message words from H for the second injection instead of keeping them live across E8
// (16 fewer VGPRs; variant measured by tools/x11_variants.hip).
template <bool kReload = false>
__device__ __forceinline__ void jh512_64(u64 h[8], const u32 (*BC)[8], const u64* __restrict__ Hb = nullptr,
                                         u32 stride = 0, u32 i = 0) {
  u32 m[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) { m[2 * k] = lo32(h[k]); m[2 * k + 1] = hi32(h[k]); }
  u32 x[8][4];
#pragma unroll
  for (int k = 0; k < 32; ++k) x[k / 4][k % 4] = x11t::JH_IV[k];
#pragma unroll
  for (int k = 0; k < 16; ++k) x[k / 4][k % 4] ^= m[k];
  jh_E8(x, BC);
  if (kReload) {
    u64 r[8];
    load_hash(Hb, stride, i, r);
#pragma unroll
    for (int k = 0; k < 8; ++k) { m[2 * k] = lo32(r[k]); m[2 * k + 1] = hi32(r[k]); }
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) x[4 + k / 4][k % 4] ^= m[k];
  // padding block: 0x80, zeros, 128-bit big-endian bit length (512)
  x[0][0] ^= 0x80u;
  x[3][3] ^= 0x00020000u;
  jh_E8(x, BC);
  x[4][0] ^= 0x80u;
  x[7][3] ^= 0x00020000u;
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = mk64(x[4 + k / 2][2 * (k % 2)], x[4 + k / 2][2 * (k % 2) + 1]);
}

// ------------------------------------------------------------------ Keccak-512
__constant__ u64 c_keccak_rc[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
constexpr int kKeccakRot[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

__device__ __forceinline__ u64 rotl64z(u64 x, int n) { return n == 0 ? x : rotl64(x, n); }

// chi: a ^ (~b & c) in one v_bitop3 per 32-bit half.
__device__ __forceinline__ u64 keccak_chi(u64 a, u64 b, u64 c) {
  return mk64(bop3<0xD2>(lo32(a), lo32(b), lo32(c)), bop3<0xD2>(hi32(a), hi32(b), hi32(c)));
}
__device__ __forceinline__ u64 xor5_64(u64 a, u64 b, u64 c, u64 d, u64 e) { return xor3_64(xor3_64(a, b, c), d, e); }

__device__ __forceinline__ void keccak512_64(u64 h[8]) {
  u64 A[25];
#pragma unroll
  for (int k = 0; k < 8; ++k) A[k] = h[k];
  A[8] = 0x8000000000000001ull;  // pad 0x01 at byte 64, 0x80 at byte 71 (rate 72)
#pragma unroll
  for (int k = 9; k < 25; ++k) A[k] = 0;
#pragma unroll 1
  for (int r = 0; r < 24; ++r) {
    u64 C[5], D[5], B[25];
#pragma unroll
    for (int x = 0; x < 5; ++x) C[x] = xor5_64(A[x], A[x + 5], A[x + 10], A[x + 15], A[x + 20]);
#pragma unroll
    for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ rotl64(C[(x + 1) % 5], 1);
#pragma unroll
    for (int x = 0; x < 5; ++x)
#pragma unroll
      for (int y = 0; y < 5; ++y) B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(A[x + 5 * y] ^ D[x], kKeccakRot[x + 5 * y]);
#pragma unroll
    for (int x = 0; x < 5; ++x)
#pragma unroll
      for (int y = 0; y < 5; ++y) A[x + 5 * y] = keccak_chi(B[x + 5 * y], B[(x + 1) % 5 + 5 * y], B[(x + 2) % 5 + 5 * y]);
    A[0] ^= c_keccak_rc[r];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = A[k];
}

// ------------------------------------------------------------------ Luffa-512
constexpr u32 kLuffaIv[5][8] = {
    {0x6d251e69, 0x44b051e0, 0x4eaa6fb4, 0xdbf78465, 0x6e292011, 0x90152df4, 0xee058139, 0xdef610bb},
    {0xc3b44b95, 0xd9d2f256, 0x70eee9a0, 0xde099fa3, 0x5d9b0557, 0x8fc944b3, 0xcf1ccf0e, 0x746cd581},
    {0xf7efc89d, 0x5dba5781, 0x04016ce5, 0xad659c05, 0x0306194f, 0x666d1836, 0x24aa230a, 0x8b264ae7},
    {0x858075d5, 0x36d79cce, 0xe571f7d7, 0x204b1f67, 0x35870c6a, 0x57e9e923, 0x14bcb808, 0x7cde72ce},
    {0x6c68e9be, 0x5ec41e22, 0xc825b7c7, 0xaffb4363, 0xf5df3999, 0x0fc688f1, 0xb07224cc, 0x03e86cea}};
constexpr u32 kLuffaRc0[5][8] = {
    {0x303994a6, 0xc0e65299, 0x6cc33a12, 0xdc56983e, 0x1e00108f, 0x7800423d, 0x8f5b7882, 0x96e1db12},
    {0xb6de10ed, 0x70f47aae, 0x0707a3d4, 0x1c1e8f51, 0x707a3d45, 0xaeb28562, 0xbaca1589, 0x40a46f3e},
    {0xfc20d9d2, 0x34552e25, 0x7ad8818f, 0x8438764a, 0xbb6de032, 0xedb780c8, 0xd9847356, 0xa2c78434},
    {0xb213afa5, 0xc84ebe95, 0x4e608a22, 0x56d858fe, 0x343b138f, 0xd0ec4e3d, 0x2ceb4882, 0xb3ad2208},
    {0xf0d2e9e3, 0xac11d7fa, 0x1bcb66f2, 0x6f2d9bc9, 0x78602649, 0x8edae952, 0x3b6ba548, 0xedae9520}};
constexpr u32 kLuffaRc4[5][8] = {
    {0xe0337818, 0x441ba90d, 0x7f34d442, 0x9389217f, 0xe5a8bce6, 0x5274baf4, 0x26889ba7, 0x9a226e9d},
    {0x01685f3d, 0x05a17cf4, 0xbd09caca, 0xf4272b28, 0x144ae5cc, 0xfaa7ae2b, 0x2e48f1c1, 0xb923c704},
    {0xe25e72c1, 0xe623bb72, 0x5c58a4a4, 0x1e38e2e7, 0x78e38b9d, 0x27586719, 0x36eda57f, 0x703aace7},
    {0xe028c9bf, 0x44756f91, 0x7e8fce32, 0x956548be, 0xfe191be2, 0x3cb226e5, 0x5944a28e, 0xa1c4c355},
    {0x5090d577, 0x2d1925ab, 0xb46496ac, 0xd1925ab0, 0x29131ab6, 0x0fc053c3, 0x3f014f0c, 0xfc053c31}};

// Multiplication by x in GF(2^32)[x]/(the Luffa polynomial) on a 256-bit word.
__device__ __forceinline__ void luffa_m2(u32 a[8]) {
  const u32 t = a[7];
  a[7] = a[6]; a[6] = a[5]; a[5] = a[4];
  a[4] = a[3] ^ t; a[3] = a[2] ^ t; a[2] = a[1];
  a[1] = a[0] ^ t; a[0] = t;
}
// Bitsliced SubCrumb (4-bit S-box {13,14,0,1,5,10,7,6,11,3,9,12,15,8,2,4}, a0 = bit 0) as four
// Shannon splits on a3: y_k = a3 ? g1_k(a0,a1,a2) : g0_k(a0,a1,a2), each cofactor and the select one
// v_bitop3: 12 VALU (the and/or/xor network is 16).
#define LUFFA_SUBCRUMB(a0, a1, a2, a3)                                                   \
  do {                                                                                   \
    const u32 y0_ = bop3<0xCA>(a3, bop3<0x17>(a0, a1, a2), bop3<0x4B>(a0, a1, a2));      \
    const u32 y1_ = bop3<0xCA>(a3, bop3<0x1B>(a0, a1, a2), bop3<0xB8>(a0, a1, a2));      \
    const u32 y2_ = bop3<0xCA>(a3, bop3<0xC2>(a0, a1, a2), bop3<0x9B>(a0, a1, a2));      \
    const u32 y3_ = bop3<0xCA>(a3, bop3<0x67>(a0, a1, a2), bop3<0x31>(a0, a1, a2));      \
    (a0) = y0_; (a1) = y1_; (a2) = y2_; (a3) = y3_;                                       \
  } while (0)
#define LUFFA_MIXWORD(u, v)          \
  do {                               \
    (v) ^= (u);                      \
    (u) = rotl32((u), 2) ^ (v);      \
    (v) = rotl32((v), 14) ^ (u);     \
    (u) = rotl32((u), 10) ^ (v);     \
    (v) = rotl32((v), 1);            \
  } while (0)

template <int J>
__device__ __forceinline__ void luffa_Q(u32 a[8]) {
#pragma unroll
  for (int k = 4; k < 8; ++k) a[k] = rotl32(a[k], J);
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    LUFFA_SUBCRUMB(a[0], a[1], a[2], a[3]);
    LUFFA_SUBCRUMB(a[5], a[6], a[7], a[4]);
#pragma unroll
    for (int k = 0; k < 4; ++k) LUFFA_MIXWORD(a[k], a[k + 4]);
    a[0] ^= kLuffaRc0[J][r];
    a[4] ^= kLuffaRc4[J][r];
  }
}

// Message injection MI5 followed by the five sub-permutations Q_j.
__device__ __forceinline__ void luffa_round(u32 V[5][8], const u32 Min[8]) {
  u32 t[8], M[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { M[k] = Min[k]; t[k] = V[0][k] ^ V[1][k] ^ V[2][k] ^ V[3][k] ^ V[4][k]; }
  luffa_m2(t);
#pragma unroll
  for (int j = 0; j < 5; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) V[j][k] ^= t[k];
#pragma unroll
  for (int k = 0; k < 8; ++k) t[k] = V[0][k];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    luffa_m2(V[j]);
#pragma unroll
    for (int k = 0; k < 8; ++k) V[j][k] ^= (j < 4 ? V[j + 1][k] : t[k]);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) t[k] = V[4][k];
#pragma unroll
  for (int j = 4; j >= 0; --j) {
    luffa_m2(V[j]);
#pragma unroll
    for (int k = 0; k < 8; ++k) V[j][k] ^= (j > 0 ? V[j - 1][k] : t[k]);
  }
#pragma unroll
  for (int j = 0; j < 5; ++j) {
#pragma unroll
    for (int k = 0; k < 8; ++k) V[j][k] ^= M[k];
    if (j < 4) luffa_m2(M);
  }
  luffa_Q<0>(V[0]);
  luffa_Q<1>(V[1]);
  luffa_Q<2>(V[2]);
  luffa_Q<3>(V[3]);
  luffa_Q<4>(V[4]);
}

__device__ __forceinline__ void luffa512_64(u64 h[8]) {
  u32 V[5][8];
#pragma unroll
  for (int j = 0; j < 5; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) V[j][k] = kLuffaIv[j][k];
  // Five rounds: two message blocks (big-endian words), the padding block, two blank
  // output rounds. Rolled: each round is ~3k instructions.
#pragma unroll 1
  for (int b = 0; b < 5; ++b) {
    u32 M[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u64 w = b == 0 ? h[k] : h[4 + k];
      M[2 * k] = b < 2 ? bswap32(lo32(w)) : 0u;
      M[2 * k + 1] = b < 2 ? bswap32(hi32(w)) : 0u;
    }
    if (b == 2) M[0] = 0x80000000u;
    luffa_round(V, M);
    if (b >= 3) {
      u32 o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = bswap32(V[0][k] ^ V[1][k] ^ V[2][k] ^ V[3][k] ^ V[4][k]);
      if (b == 3) {
#pragma unroll
        for (int k = 0; k < 4; ++k) h[k] = mk64(o[2 * k], o[2 * k + 1]);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) h[4 + k] = mk64(o[2 * k], o[2 * k + 1]);
      }
    }
  }
}
#undef LUFFA_SUBCRUMB
#undef LUFFA_MIXWORD

// ------------------------------------------------------------------ CubeHash-512
// One round; the word swaps are register renames once two rounds are unrolled
// (the round's permutation is an involution).
__device__ __forceinline__ void cube_round(u32 x[32]) {
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i + 16] += x[i];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = rotl32(x[i], 7);
#pragma unroll
  for (int i = 0; i < 8; ++i) { const u32 t = x[i]; x[i] = x[i + 8]; x[i + 8] = t; }
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] ^= x[i + 16];
#pragma unroll
  for (int i = 16; i < 32; ++i)
    if (!(i & 2)) { const u32 t = x[i]; x[i] = x[i + 2]; x[i + 2] = t; }
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i + 16] += x[i];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = rotl32(x[i], 11);
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (!(i & 4)) { const u32 t = x[i]; x[i] = x[i + 4]; x[i + 4] = t; }
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] ^= x[i + 16];
#pragma unroll
  for (int i = 16; i < 32; ++i)
    if (!(i & 1)) { const u32 t = x[i]; x[i] = x[i + 1]; x[i + 1] = t; }
}
__device__ __forceinline__ void cube_rounds(u32 x[32], int n) {
#pragma unroll 1
  for (int r = 0; r < n; r += 2) {
    cube_round(x);
    cube_round(x);
  }
}

__device__ __forceinline__ void cubehash512_64(u64 h[8]) {
  u32 x[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) x[k] = x11t::CUBE_IV[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) { x[2 * k] ^= lo32(h[k]); x[2 * k + 1] ^= hi32(h[k]); }
  cube_rounds(x, 16);
#pragma unroll
  for (int k = 0; k < 4; ++k) { x[2 * k] ^= lo32(h[4 + k]); x[2 * k + 1] ^= hi32(h[4 + k]); }
  cube_rounds(x, 16);
  x[0] ^= 0x80u;  // padding block
  cube_rounds(x, 16);
  x[31] ^= 1u;    // finalization
  cube_rounds(x, 160);
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = mk64(x[2 * k], x[2 * k + 1]);
}

// One kernel per stage: each stage runs at its own register budget / occupancy.
#define X11_STAGE_KERNEL(NAME, FN)                                                                       \
  __global__ __launch_bounds__(kBlock) void NAME(u64* __restrict__ Hb, u32 stride, u32 n, X11Abort ab) { \
    const u32 i = blockIdx.x * kBlock + threadIdx.x;                                                     \
    if (i >= n) return;                                                                                  \
    const u32 a0 = x11_abort_issue(ab);                                                                  \
    u64 h[8];                                                                                            \
    load_hash(Hb, stride, i, h);                                                                         \
    if (x11_abort_seen(a0, ab)) return;                                                                  \
    FN(h);                                                                                               \
    store_hash(Hb, stride, i, h);                                                                        \
  }
X11_STAGE_KERNEL(k_bmw512_64, bmw512_64)
X11_STAGE_KERNEL(k_skein512_64, skein512_64)
X11_STAGE_KERNEL(k_keccak512_64, keccak512_64)
X11_STAGE_KERNEL(k_luffa512_64, luffa512_64)
X11_STAGE_KERNEL(k_cubehash512_64, cubehash512_64)
#undef X11_STAGE_KERNEL

__device__ __forceinline__ void jh_stage_lds(u64* __restrict__ Hb, u32 stride, u32 n, bool reload,
                                             X11Abort ab = X11Abort{}) {
  __shared__ __attribute__((aligned(16))) u32 BC[42][8];
  for (u32 t = threadIdx.x; t < 42 * 8; t += kBlock) BC[t / 8][t % 8] = x11t::JH_BC[t / 8][t % 8];
  __syncthreads();
  const u32 i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const u32 a0 = x11_abort_issue(ab);
  u64 h[8];
  load_hash(Hb, stride, i, h);
  if (x11_abort_seen(a0, ab)) return;
  if (reload) jh512_64<true>(h, BC, Hb, stride, i);
  else jh512_64(h, BC);
  store_hash(Hb, stride, i, h);
}
// Round constants staged in LDS so each round's eight words arrive in VGPRs by ds_read (from the scalar cache
// they need one v_mov per word: 672 per hash, 5.5% of JH's VALU), the message re-read from H for the second
// injection, 7 waves/SIMD (72 VGPRs, 44 B of spills outside the round loops). Same-run times per 2^23 against
// the scalar-cache kernel in four sessions: -4.4%, -2.0%, -1.3%, +1.0% (tools/x11_variants.hip,
// profiles/r3/h_jh, l_shavite, x_simd).
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(7, 8))) void k_jh512_64(
    u64* __restrict__ Hb, u32 stride, u32 n, X11Abort ab) {
  jh_stage_lds(Hb, stride, n, true, ab);
}
#ifdef OTEDAMA_X11_VARIANTS
// Alternatives timed by tools/x11_variants.hip (not built into the extension).
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(7, 8))) void k_jh512_64_w7(
    u64* __restrict__ Hb, u32 stride, u32 n) {
  jh_stage_lds(Hb, stride, n, false);
}
__global__ __launch_bounds__(kBlock) void k_jh512_64_sgpr(u64* __restrict__ Hb, u32 stride, u32 n) {
  const u32 i = blockIdx.x * kBlock + threadIdx.x;  // round constants through the scalar cache + v_mov
  if (i >= n) return;
  u64 h[8];
  load_hash(Hb, stride, i, h);
  jh512_64(h, x11t::JH_BC);
  store_hash(Hb, stride, i, h);
}
__global__ __launch_bounds__(kBlock) void k_jh512_64_lds(u64* __restrict__ Hb, u32 stride, u32 n) {
  jh_stage_lds(Hb, stride, n, false);
}
#endif

__global__ __launch_bounds__(kBlock) void k_blake512_80(X11Params p, u32 base, u64* __restrict__ H, u32 stride, u32 n,
                                                       X11Abort ab) {
  const u32 i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n || x11_stop(ab)) return;
  u64 h[8];
  blake512_80(p, base + i, h);
  store_hash(H, stride, i, h);
}
}  // namespace x11k

hipError_t x11_launch_stage_a(int stage, const X11Params& p, uint32_t base, uint64_t* H, uint32_t stride, uint32_t n,
                              X11Abort ab, hipStream_t s) {
  using namespace x11k;
  const dim3 grid((n + kBlock - 1) / kBlock), block(kBlock);
  const X11Abort mid = x11_midstage_polls() ? ab : X11Abort{};
  switch (stage) {
    case kX11Blake: k_blake512_80<<<grid, block, 0, s>>>(p, base, H, stride, n, ab); break;
    case kX11Bmw: k_bmw512_64<<<grid, block, 0, s>>>(H, stride, n, mid); break;
    case kX11Groestl: {
      const u32 want = (n + kGroestlBlock - 1) / kGroestlBlock, cap = (u32)x11_device_cus() * 2 * 4;
      k_groestl512_64<<<dim3(want < cap ? want : cap), dim3(kGroestlBlock), 0, s>>>(H, stride, n, mid);
      break;
    }
    case kX11Skein: k_skein512_64<<<grid, block, 0, s>>>(H, stride, n, mid); break;
    case kX11Jh: k_jh512_64<<<grid, block, 0, s>>>(H, stride, n, mid); break;
    case kX11Keccak: k_keccak512_64<<<grid, block, 0, s>>>(H, stride, n, mid); break;
    case kX11Luffa: k_luffa512_64<<<grid, block, 0, s>>>(H, stride, n, mid); break;
    case kX11Cubehash: k_cubehash512_64<<<grid, block, 0, s>>>(H, stride, n, mid); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace otedama
