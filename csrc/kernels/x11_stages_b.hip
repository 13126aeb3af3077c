// X11 stages 9-11 on gfx950: SHAvite-3-512, SIMD-512, ECHO-512 (all on the 64-byte
// output of the previous stage), plus the chain launcher and the target compare fused
// into the ECHO stage.
//
// SHAvite / ECHO: one lane per nonce. The padding blocks of
// the fixed 64-byte inputs are folded into constants (SHAvite and ECHO are a
// single compression; their counters are the constant 512).
// SIMD: eight lanes per nonce. Lane j owns NTT columns 2j and 2j+1, which are
// exactly the coefficients its message words W[.][j] are built from, so the
// 256-point NTT and the expansion need no lane exchange; the 36 Feistel steps
// keep state column j in lane j and exchange one word per step with an xor
// shuffle inside the 8-lane group.
// Bit-exact oracle: csrc/cpu/x11_cpu.cpp (tests/test_x11_gpu.py compares every stage).
#include <cstdlib>

#include "otedama/x11_launch.h"
#include "x11_common.h"

namespace otedama {
namespace x11k {

// ------------------------------------------------------------------ SHAvite-3-512
constexpr u32 kShaviteIv[16] = {0x72FCCDD8, 0x79CA4727, 0x128A077B, 0x40D55AEC, 0xD1901A06, 0x430AE307,
                                0xB29F5CD1, 0xDF07FBFC, 0x8E45D73D, 0x681AB538, 0xBDE86578, 0xDD577E47,
                                0xE275EADE, 0x502D9FCD, 0xB9357178, 0x022A4B9A};

// F: four AES rounds, round key i added before round i; keys 1..3 ride in the previous round's
// output xor3.
constexpr int kAesBlock = 512;
__device__ __forceinline__ void shavite_F(const u32* T, u32 lo, u32 x[4], const u32* k) {
  x[0] ^= k[0]; x[1] ^= k[1]; x[2] ^= k[2]; x[3] ^= k[3];
  aes_round_k(T, lo, x[0], x[1], x[2], x[3], k[4], k[5], k[6], k[7]);
  aes_round_k(T, lo, x[0], x[1], x[2], x[3], k[8], k[9], k[10], k[11]);
  aes_round_k(T, lo, x[0], x[1], x[2], x[3], k[12], k[13], k[14], k[15]);
  aes_round(T, lo, x[0], x[1], x[2], x[3]);
}

// Key schedule, odd rounds: the AES-based step on the rolling 32-word window. The counter {512, 0, 0, 0} enters at
// rounds 1, 5, 9, 13 (kInj 0..3), right after the word group that the spec mixes it into.
template <int kInj>
__device__ __forceinline__ void shavite_rk_odd(const u32* T, u32 lo, u32 rk[32]) {
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    u32 t0 = rk[4 * g + 1], t1 = rk[4 * g + 2], t2 = rk[4 * g + 3], t3 = rk[4 * g];
    aes_round(T, lo, t0, t1, t2, t3);
    const int p = g ? 4 * g - 4 : 28;
    rk[4 * g] = t0 ^ rk[p];
    rk[4 * g + 1] = t1 ^ rk[p + 1];
    rk[4 * g + 2] = t2 ^ rk[p + 2];
    rk[4 * g + 3] = t3 ^ rk[p + 3];
    if (kInj == 0 && g == 0) { rk[0] ^= 512u; rk[3] = ~rk[3]; }
    if (kInj == 1 && g == 1) { rk[7] ^= ~512u; }
    if (kInj == 2 && g == 7) { rk[30] ^= 512u; rk[31] = ~rk[31]; }
    if (kInj == 3 && g == 6) { rk[25] ^= 512u; rk[27] = ~rk[27]; }
  }
}
// Key schedule, even rounds: rk[i] = rk[i - 32] ^ rk[i - 7] on the window.
__device__ __forceinline__ void shavite_rk_even(u32 rk[32]) {
#pragma unroll
  for (int k = 0; k < 32; ++k) rk[k] ^= k >= 7 ? rk[k - 7] : rk[k + 25];
}
// One round on the state (a, b, c, d): a ^= F(b, rk[0..15]), c ^= F(d, rk[16..31]); the next round's state is
// (d, a, b, c), which the caller realises by passing the arrays in that order (no register moves).
__device__ __forceinline__ void shavite_round(const u32* T, u32 lo, const u32 rk[32], u32 a[4], const u32 b[4],
                                              u32 c[4], const u32 d[4]) {
  u32 x[4] = {b[0], b[1], b[2], b[3]};
  shavite_F(T, lo, x, rk);
#pragma unroll
  for (int k = 0; k < 4; ++k) a[k] ^= x[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) x[k] = d[k];
  shavite_F(T, lo, x, rk + 16);
#pragma unroll
  for (int k = 0; k < 4; ++k) c[k] ^= x[k];
}

// 14 rounds: round 0, three trips of rounds 4t+1 .. 4t+4 (odd, even, odd, even: the state rotation closes after
// four rounds, so the rolled loop carries no register moves), round 13. The one-round rolled loop it replaces spent
// ~85 v_mov per round on the rotation and the schedule window (18% of SHAvite's VALU; tools/x11_variants.hip).
__device__ __forceinline__ void shavite512_64(const u32* T, u32 lo, u64 h[8]) {
  // Rolling 32-word window of the 448-word key schedule; block 0 is the padded message.
  u32 rk[32];
#pragma unroll
  for (int k = 0; k < 8; ++k) { rk[2 * k] = lo32(h[k]); rk[2 * k + 1] = hi32(h[k]); }
  rk[16] = 0x80u;
#pragma unroll
  for (int k = 17; k < 32; ++k) rk[k] = 0;
  rk[27] = 0x02000000u;  // 512-bit length at bytes 110..113
  rk[31] = 0x02000000u;  // digest size 512 at bytes 126..127
  u32 A[4], B[4], C[4], D[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    A[k] = kShaviteIv[k]; B[k] = kShaviteIv[4 + k]; C[k] = kShaviteIv[8 + k]; D[k] = kShaviteIv[12 + k];
  }
  shavite_round(T, lo, rk, A, B, C, D);  // round 0: the message block itself
#pragma unroll 1
  for (int t = 0; t < 3; ++t) {
    if (t == 0) shavite_rk_odd<0>(T, lo, rk);
    else if (t == 1) shavite_rk_odd<1>(T, lo, rk);
    else shavite_rk_odd<2>(T, lo, rk);
    shavite_round(T, lo, rk, D, A, B, C);
    shavite_rk_even(rk);
    shavite_round(T, lo, rk, C, D, A, B);
    shavite_rk_odd<-1>(T, lo, rk);
    shavite_round(T, lo, rk, B, C, D, A);
    shavite_rk_even(rk);
    shavite_round(T, lo, rk, A, B, C, D);
  }
  shavite_rk_odd<3>(T, lo, rk);
  shavite_round(T, lo, rk, D, A, B, C);
  // the state after round 13 is (C, D, A, B) in the spec's order
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const u32 a = C[k], b = D[k];
    C[k] = A[k]; D[k] = B[k]; A[k] = a; B[k] = b;
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    h[k] = mk64(kShaviteIv[2 * k] ^ A[2 * k], kShaviteIv[2 * k + 1] ^ A[2 * k + 1]);
    h[2 + k] = mk64(kShaviteIv[4 + 2 * k] ^ B[2 * k], kShaviteIv[5 + 2 * k] ^ B[2 * k + 1]);
    h[4 + k] = mk64(kShaviteIv[8 + 2 * k] ^ C[2 * k], kShaviteIv[9 + 2 * k] ^ C[2 * k + 1]);
    h[6 + k] = mk64(kShaviteIv[12 + 2 * k] ^ D[2 * k], kShaviteIv[13 + 2 * k] ^ D[2 * k + 1]);
  }
}

__device__ __forceinline__ void shavite_stage(u64* __restrict__ Hb, u32 stride, u32 n, X11Abort ab) {
  __shared__ u32 T[kAesPrivWords];
  aes_priv_fill(T);
  const u32 lo = aes_laneoff();
  for (u32 i = blockIdx.x * kAesBlock + threadIdx.x; i < n; i += gridDim.x * kAesBlock) {
    const u32 a0 = x11_abort_issue(ab);
    u64 h[8];
    load_hash(Hb, stride, i, h);
    if (x11_abort_seen(a0, ab)) return;
    shavite512_64(T, lo, h);
    store_hash(Hb, stride, i, h);
  }
}
__global__ __launch_bounds__(kAesBlock) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_shavite512_64(
    u64* __restrict__ Hb, u32 stride, u32 n, X11Abort ab) {
  shavite_stage(Hb, stride, n, ab);
}
#ifdef OTEDAMA_X11_VARIANTS
// The round-2 kernel, verbatim (one round per trip of a rolled loop), timed by tools/x11_variants.hip.
__global__ __launch_bounds__(kAesBlock) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_shavite512_64_r2(u64* __restrict__ Hb, u32 stride, u32 n) {
  __shared__ u32 T[kAesPrivWords];
  aes_priv_fill(T);
  const u32 lo = aes_laneoff();
  for (u32 i = blockIdx.x * kAesBlock + threadIdx.x; i < n; i += gridDim.x * kAesBlock) {
  u64 h[8];
  load_hash(Hb, stride, i, h);
  // Rolling 32-word window of the 448-word key schedule; block 0 is the padded message.
  u32 rk[32];
#pragma unroll
  for (int k = 0; k < 8; ++k) { rk[2 * k] = lo32(h[k]); rk[2 * k + 1] = hi32(h[k]); }
  rk[16] = 0x80u;
#pragma unroll
  for (int k = 17; k < 32; ++k) rk[k] = 0;
  rk[27] = 0x02000000u;  // 512-bit length at bytes 110..113
  rk[31] = 0x02000000u;  // digest size 512 at bytes 126..127
  u32 A[4], B[4], C[4], D[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    A[k] = kShaviteIv[k]; B[k] = kShaviteIv[4 + k]; C[k] = kShaviteIv[8 + k]; D[k] = kShaviteIv[12 + k];
  }
  // counter = {512, 0, 0, 0}
#pragma unroll 1
  for (int r = 0; r < 14; ++r) {
    if (r & 1) {
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        u32 t0 = rk[4 * g + 1], t1 = rk[4 * g + 2], t2 = rk[4 * g + 3], t3 = rk[4 * g];
        aes_round(T, lo, t0, t1, t2, t3);
        const int p = g ? 4 * g - 4 : 28;
        rk[4 * g] = t0 ^ rk[p];
        rk[4 * g + 1] = t1 ^ rk[p + 1];
        rk[4 * g + 2] = t2 ^ rk[p + 2];
        rk[4 * g + 3] = t3 ^ rk[p + 3];
        if (g == 0 && r == 1) { rk[0] ^= 512u; rk[3] = ~rk[3]; }
        if (g == 1 && r == 5) { rk[7] ^= ~512u; }
        if (g == 7 && r == 9) { rk[30] ^= 512u; rk[31] = ~rk[31]; }
        if (g == 6 && r == 13) { rk[25] ^= 512u; rk[27] = ~rk[27]; }
      }
    } else if (r) {
#pragma unroll
      for (int k = 0; k < 32; ++k) rk[k] ^= k >= 7 ? rk[k - 7] : rk[k + 25];
    }
    u32 x[4] = {B[0], B[1], B[2], B[3]};
    shavite_F(T, lo, x, rk);
#pragma unroll
    for (int k = 0; k < 4; ++k) A[k] ^= x[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = D[k];
    shavite_F(T, lo, x, rk + 16);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      C[k] ^= x[k];
      const u32 t = D[k];
      D[k] = C[k]; C[k] = B[k]; B[k] = A[k]; A[k] = t;
    }
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    h[k] = mk64(kShaviteIv[2 * k] ^ A[2 * k], kShaviteIv[2 * k + 1] ^ A[2 * k + 1]);
    h[2 + k] = mk64(kShaviteIv[4 + 2 * k] ^ B[2 * k], kShaviteIv[5 + 2 * k] ^ B[2 * k + 1]);
    h[4 + k] = mk64(kShaviteIv[8 + 2 * k] ^ C[2 * k], kShaviteIv[9 + 2 * k] ^ C[2 * k + 1]);
    h[6 + k] = mk64(kShaviteIv[12 + 2 * k] ^ D[2 * k], kShaviteIv[13 + 2 * k] ^ D[2 * k + 1]);
  }
  store_hash(Hb, stride, i, h);
  }
}
#endif

// ------------------------------------------------------------------ SIMD-512
constexpr u32 kSimdIv[32] = {
    0x0BA16B95, 0x72F999AD, 0x9FECC2AE, 0xBA3264FC, 0x5E894929, 0x8E9F30E5, 0x2F1DAA37, 0xF0F2C558,
    0xAC506643, 0xA90635A5, 0xE25B878B, 0xAAB7878F, 0x88817F7A, 0x0A02892B, 0x559A7550, 0x598F657E,
    0x7EEF60A1, 0x6B70E3E8, 0x9C1714D1, 0xB958E2A8, 0xAB02675E, 0xED1C014F, 0xCD8D65BB, 0xFDB7A257,
    0x09254899, 0xD699C7BC, 0x9019B6DC, 0x2B9022E4, 0x8FA14956, 0x21BF9BD3, 0xB94D0943, 0x6FFDDC22};
constexpr int kSimdPP[7] = {1, 6, 2, 3, 5, 7, 4};
constexpr int kSimdRS[4][4] = {{3, 23, 17, 27}, {28, 19, 22, 7}, {29, 9, 15, 5}, {4, 13, 10, 25}};
constexpr int kSimdSB[32] = {4, 6, 0, 2, 7, 5, 3, 1, 15, 11, 12, 8, 9, 13, 10, 14,
                             17, 18, 23, 20, 22, 21, 16, 19, 30, 24, 25, 31, 27, 29, 28, 26};

// Column b of the first-block NTT (see tools/gen_x11_tables.cpp, which checks this exact integer
// form against the direct transform): u_d = dot4(X_d, PT[b][d]) + S_d with X_d = bytes x[16c+d]
// (c = 0..3) and PT[b][d] byte c = alpha^(b(16c+d)) - 1, so one v_dot4_u32_u8 per coefficient;
// then the 16-point DFT with root 2 as 4 x 4 with root 16 (shifts and adds only), the first-block
// twiddle beta_b 2^-a, and a centred reduction mod 257.
__device__ __forceinline__ int fold257(int x) { return (x & 255) - (x >> 8); }
__device__ __forceinline__ int centre257(int x) {
  x = fold257(fold257(fold257(x)));  // |x| < 2^27 -> [-8, 264]
  return x > 128 ? x - 257 : x;
}
template <int E>
__device__ __forceinline__ int mul2pow(int x) {
  constexpr int e = ((E % 16) + 16) % 16;
  if constexpr (e < 8) return x << e;
  else return -(x << (e - 8));
}
__device__ __forceinline__ void dft4_16(int i0, int i1, int i2, int i3, int& o0, int& o1, int& o2, int& o3) {
  const int e0 = i0 + i2, e1 = i0 - i2, p0 = i1 + i3, p1 = i1 - i3;
  o0 = e0 + p0; o2 = e0 - p0; o1 = e1 + (p1 << 4); o3 = e1 - (p1 << 4);
}
__device__ __forceinline__ void simd_ntt_column(const u32 X[16], const u32 S[16], const u32* PT, int beta, int q[16]) {
  int u[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) u[d] = fold257((int)__builtin_amdgcn_udot4(X[d], PT[d], S[d], false));
  int W[4][4];
#pragma unroll
  for (int d1 = 0; d1 < 4; ++d1) {
    int v0, v1, v2, v3;
    dft4_16(u[d1], u[4 + d1], u[8 + d1], u[12 + d1], v0, v1, v2, v3);
    W[d1][0] = v0;
    W[d1][1] = d1 == 0 ? v1 : d1 == 1 ? mul2pow<1>(v1) : d1 == 2 ? mul2pow<2>(v1) : mul2pow<3>(v1);
    W[d1][2] = d1 == 0 ? v2 : d1 == 1 ? mul2pow<2>(v2) : d1 == 2 ? mul2pow<4>(v2) : mul2pow<6>(v2);
    W[d1][3] = d1 == 0 ? v3 : d1 == 1 ? mul2pow<3>(v3) : d1 == 2 ? mul2pow<6>(v3) : mul2pow<9>(v3);
  }
#pragma unroll
  for (int a1 = 0; a1 < 4; ++a1) {
    int y0, y1, y2, y3;
    dft4_16(W[0][a1], W[1][a1], W[2][a1], W[3][a1], y0, y1, y2, y3);
    q[a1] = centre257(y0 + (a1 == 0 ? beta : a1 == 1 ? mul2pow<15>(beta) : a1 == 2 ? mul2pow<14>(beta) : mul2pow<13>(beta)));
    q[a1 + 4] = centre257(y1 + (a1 == 0 ? mul2pow<12>(beta) : a1 == 1 ? mul2pow<11>(beta) : a1 == 2 ? mul2pow<10>(beta) : mul2pow<9>(beta)));
    q[a1 + 8] = centre257(y2 + (a1 == 0 ? mul2pow<8>(beta) : a1 == 1 ? mul2pow<7>(beta) : a1 == 2 ? mul2pow<6>(beta) : mul2pow<5>(beta)));
    q[a1 + 12] = centre257(y3 + (a1 == 0 ? mul2pow<4>(beta) : a1 == 1 ? mul2pow<3>(beta) : a1 == 2 ? mul2pow<2>(beta) : mul2pow<1>(beta)));
  }
}

// tA of lane j ^ PP inside the 8-lane group. xor 1/2/3 by DPP quad_perm and xor 7 by DPP row_half_mirror: the
// compiler fuses those into the consuming add. xor 4/5/6 have no single DPP pattern (as DPP they cost a
// separate v_mov_dpp, 31 VALU per lane over the two compressions); ds_swizzle's bit-mask mode reads lane
// (l & 0x1F) ^ PP on the LDS unit instead, off the VALU, issued as soon as tA exists.
template <int PP, bool kSw = true>
__device__ __forceinline__ u32 simd_xlane(u32 v) {
  if constexpr (!kSw && PP >= 4 && PP <= 6) {  // round-2 form (tools/x11_variants.hip): xor 7, then xor 3/2/1
    v = (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    constexpr int q = PP == 6 ? 0xB1 : PP == 5 ? 0x4E : 0x1B;
    return (u32)__builtin_amdgcn_update_dpp(0, (int)v, q, 0xF, 0xF, false);
  } else if constexpr (PP >= 4 && PP <= 6) {
    return (u32)__builtin_amdgcn_ds_swizzle((int)v, (PP << 10) | 0x1F);
  } else if constexpr (PP == 7) {
    return (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror: xor 7
  } else {
    constexpr int q = PP == 1 ? 0xB1 : PP == 2 ? 0x4E : 0x1B;  // quad_perm: xor 1 / 2 / 3
    return (u32)__builtin_amdgcn_update_dpp(0, (int)v, q, 0xF, 0xF, false);
  }
}

// One Feistel step on state column j (this lane).
template <bool kMaj, int R, int S, int PP, bool kSw = true>
__device__ __forceinline__ void simd_step(u32& s0, u32& s1, u32& s2, u32& s3, u32 w) {
  const u32 tA = rotl32(s0, R);
  const u32 f = kMaj ? bop3<0xE8>(s0, s1, s2) : bop3<0xCA>(s0, s1, s2);  // MAJ / IF
  const u32 tt = s3 + w + f;
  s0 = rotl32(tt, S) + simd_xlane<PP, kSw>(tA);
  s3 = s2;
  s2 = s1;
  s1 = tA;
}

template <int RD, bool kSw = true>
__device__ __forceinline__ void simd_round(u32& s0, u32& s1, u32& s2, u32& s3, const u32 w[8]) {
  constexpr int r0 = kSimdRS[RD][0], r1 = kSimdRS[RD][1], r2 = kSimdRS[RD][2], r3 = kSimdRS[RD][3];
  simd_step<false, r0, r1, kSimdPP[(0 + RD) % 7], kSw>(s0, s1, s2, s3, w[0]);
  simd_step<false, r1, r2, kSimdPP[(1 + RD) % 7], kSw>(s0, s1, s2, s3, w[1]);
  simd_step<false, r2, r3, kSimdPP[(2 + RD) % 7], kSw>(s0, s1, s2, s3, w[2]);
  simd_step<false, r3, r0, kSimdPP[(3 + RD) % 7], kSw>(s0, s1, s2, s3, w[3]);
  simd_step<true, r0, r1, kSimdPP[(4 + RD) % 7], kSw>(s0, s1, s2, s3, w[4]);
  simd_step<true, r1, r2, kSimdPP[(5 + RD) % 7], kSw>(s0, s1, s2, s3, w[5]);
  simd_step<true, r2, r3, kSimdPP[(6 + RD) % 7], kSw>(s0, s1, s2, s3, w[6]);
  simd_step<true, r3, r0, kSimdPP[(7 + RD) % 7], kSw>(s0, s1, s2, s3, w[7]);
}

// 32 message steps + 4 feed-forward steps; h0..h3 = chaining column, s0..s3 = h ^ block.
template <bool kSw = true>
__device__ __forceinline__ void simd_compress(u32& s0, u32& s1, u32& s2, u32& s3, u32 h0, u32 h1, u32 h2, u32 h3,
                                              const u32 W[32]) {
  simd_round<0, kSw>(s0, s1, s2, s3, W);
  simd_round<1, kSw>(s0, s1, s2, s3, W + 8);
  simd_round<2, kSw>(s0, s1, s2, s3, W + 16);
  simd_round<3, kSw>(s0, s1, s2, s3, W + 24);
  simd_step<false, 4, 13, kSimdPP[4], kSw>(s0, s1, s2, s3, h0);
  simd_step<false, 13, 10, kSimdPP[5], kSw>(s0, s1, s2, s3, h1);
  simd_step<false, 10, 25, kSimdPP[6], kSw>(s0, s1, s2, s3, h2);
  simd_step<false, 25, 4, kSimdPP[0], kSw>(s0, s1, s2, s3, h3);
}

// W = (l * mm mod 2^16) | (h * mm mod 2^16) << 16: pack (l, h) as u16 halves (one v_perm), then one
// packed 16-bit multiply.
__device__ __forceinline__ u32 simd_inner(int l, int h, unsigned short mm) {
  const u32 lh = __builtin_amdgcn_perm((u32)h, (u32)l, 0x05040100u);
  return __builtin_bit_cast(u32, __builtin_bit_cast(u16x2, lh) * (u16x2)(mm));
}

// Per-block LDS tables (dwords): for lane column pair j, PT[2j][0..15] PT[2j+1][0..15] at 36j (row
// stride 36 keeps the 8 distinct rows of a ds_read_b128 lane group on distinct banks); final-block
// words W_F[st][j] at 288 + 36j; SIMD IV at 576; beta_b at 608.
constexpr int kSimdBlock = 256;
constexpr u32 kSimdLds = 624;

// Eight lanes per hash: launch with 8 * n threads.
template <bool kSw>
__device__ __forceinline__ void simd_stage(u64* __restrict__ Hb, u32 stride, u32 n, X11Abort ab = X11Abort{}) {
  __shared__ __attribute__((aligned(16))) u32 L[kSimdLds];
  for (u32 t = threadIdx.x; t < kSimdLds; t += kSimdBlock) {
    u32 v = 0;
    if (t < 288) {
      const u32 jj = t / 36, k = t % 36;
      v = k < 16 ? x11t::SIMD_PT[2 * jj][k] : k < 32 ? x11t::SIMD_PT[2 * jj + 1][k - 16] : 0u;
    } else if (t < 576) {
      const u32 jj = (t - 288) / 36, k = (t - 288) % 36;
      v = k < 32 ? x11t::SIMD_WF[k][jj] : 0u;
    } else if (t < 608) {
      v = kSimdIv[t - 576];
    } else {
      v = x11t::SIMD_BETA[t - 608];
    }
    L[t] = v;
  }
  __syncthreads();
  const u32 t = blockIdx.x * kSimdBlock + threadIdx.x;
  const u32 i = t >> 3, j = t & 7;
  if (i >= n) return;  // whole 8-lane groups exit together
  const u32 a0 = x11_abort_issue(ab);
  u64 h[8];
  load_hash(Hb, stride, i, h);
  if (x11_abort_seen(a0, ab)) return;  // wave-uniform: whole waves (eight 8-lane groups) leave together
  u32 xw[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) { xw[2 * k] = lo32(h[k]); xw[2 * k + 1] = hi32(h[k]); }
  // X_d = (x[d], x[16 + d], x[32 + d], x[48 + d]): 4x4 byte transposes of (xw[g], xw[4+g], xw[8+g], xw[12+g])
  u32 X[16], S[16];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const u32 p01l = __builtin_amdgcn_perm(xw[4 + g], xw[g], 0x05010400u);
    const u32 p01h = __builtin_amdgcn_perm(xw[4 + g], xw[g], 0x07030602u);
    const u32 p23l = __builtin_amdgcn_perm(xw[12 + g], xw[8 + g], 0x05010400u);
    const u32 p23h = __builtin_amdgcn_perm(xw[12 + g], xw[8 + g], 0x07030602u);
    X[4 * g + 0] = __builtin_amdgcn_perm(p23l, p01l, 0x05040100u);
    X[4 * g + 1] = __builtin_amdgcn_perm(p23l, p01l, 0x07060302u);
    X[4 * g + 2] = __builtin_amdgcn_perm(p23h, p01h, 0x05040100u);
    X[4 * g + 3] = __builtin_amdgcn_perm(p23h, p01h, 0x07060302u);
  }
#pragma unroll
  for (int d = 0; d < 16; ++d) S[d] = __builtin_amdgcn_udot4(X[d], 0x01010101u, 0u, false);
  const u32* row = L + 36 * j;
  int qa[16], qb[16];
  simd_ntt_column(X, S, row, (int)L[608 + 2 * j], qa);
  simd_ntt_column(X, S, row + 16, (int)L[609 + 2 * j], qb);
  u32 W[32];
#pragma unroll
  for (int st = 0; st < 32; ++st) {
    const int sb = kSimdSB[st];
    if (st < 16) W[st] = simd_inner(qa[sb], qb[sb], 185);
    else if (st < 24) W[st] = simd_inner(qa[sb - 16], qa[sb - 8], 233);
    else W[st] = simd_inner(qb[sb - 24], qb[sb - 16], 233);
  }
  // Column j of the chaining value (IV) and of the block (message words j and 8 + j).
  const u32 iv0 = L[576 + j], iv1 = L[584 + j], iv2 = L[592 + j], iv3 = L[600 + j];
  const u32* Hw = reinterpret_cast<const u32*>(Hb);  // message words j and 8 + j (L2-resident re-read)
  const u32 m0 = Hw[((size_t)(j >> 1) * stride + i) * 2 + (j & 1)];
  const u32 m1 = Hw[((size_t)(4 + (j >> 1)) * stride + i) * 2 + (j & 1)];
  u32 s0 = iv0 ^ m0, s1 = iv1 ^ m1, s2 = iv2, s3 = iv3;
  simd_compress<kSw>(s0, s1, s2, s3, iv0, iv1, iv2, iv3, W);
  // Final block: the 512-bit length (word 0), expanded with the final tweak (constant W_F).
  const u32* wf = L + 288 + 36 * j;
#pragma unroll
  for (int st = 0; st < 32; ++st) W[st] = wf[st];
  const u32 c0 = s0, c1 = s1, c2 = s2, c3 = s3;
  if (j == 0) s0 ^= 512u;
  simd_compress<kSw>(s0, s1, s2, s3, c0, c1, c2, c3, W);
  // Output words j (s0) and 8 + j (s1); even lanes pair with their odd neighbour (DPP xor 1).
  const u32 n0 = simd_xlane<1>(s0), n1 = simd_xlane<1>(s1);
  if ((j & 1) == 0) {
    __builtin_nontemporal_store(mk64(s0, n0), Hb + (size_t)(j >> 1) * stride + i);
    __builtin_nontemporal_store(mk64(s1, n1), Hb + (size_t)(4 + (j >> 1)) * stride + i);
  }
}

__global__ __launch_bounds__(kSimdBlock) void k_simd512_64(u64* __restrict__ Hb, u32 stride, u32 n, X11Abort ab) {
  simd_stage<true>(Hb, stride, n, ab);
}
#ifdef OTEDAMA_X11_VARIANTS
__global__ __launch_bounds__(kSimdBlock) void k_simd512_64_dpp(u64* __restrict__ Hb, u32 stride, u32 n) {
  simd_stage<false>(Hb, stride, n);
}
#endif

// ------------------------------------------------------------------ ECHO-512
// GF(2^8) doubling of 4 packed bytes: the 0x1b reduction as one packed 16-bit multiply (full rate;
// a 32-bit v_mul_lo_u32 is quarter rate) and the masked shift + xor as one v_bitop3 ((a & c) ^ b).
__device__ __forceinline__ u32 xt4(u32 x) {
  const u16x2 m = __builtin_bit_cast(u16x2, (x >> 7) & 0x01010101u) * (u16x2)(0x1b);
  return bop3<0x6C>(x << 1, __builtin_bit_cast(u32, m), 0xfefefefeu);
}

// One ECHO round: BIG.SubWords (two AES rounds per 128-bit word, the first keyed by the
// running counter), BIG.ShiftRows (a renaming), BIG.MixColumns (bytewise, 4 bytes per u32).
// BIG.ShiftRows + BIG.MixColumns: column c of the row-shifted state takes row rr from column
// (c + rr) & 3; the mix is bytewise over the four 128-bit rows.
__device__ __forceinline__ void echo_mix(u32 W[16][4]) {
  u32 N[16][4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const u32 a0 = W[4 * c][w], a1 = W[4 * ((c + 1) & 3) + 1][w], a2 = W[4 * ((c + 2) & 3) + 2][w],
                a3 = W[4 * ((c + 3) & 3) + 3][w];
      const u32 ab = a0 ^ a1, bc = a1 ^ a2, cd = a2 ^ a3, da = a3 ^ a0;
      N[4 * c + 0][w] = xor3(xt4(ab), a1, cd);
      N[4 * c + 1][w] = xor3(xt4(bc), a0, cd);
      N[4 * c + 2][w] = xor3(xt4(cd), ab, a3);
      N[4 * c + 3][w] = xor3(xt4(da), a0, bc);
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int w = 0; w < 4; ++w) W[i][w] = N[i][w];
}
// BIG.SubWords of word i: two AES rounds, the first keyed by the running counter k.
__device__ __forceinline__ void echo_sub(const u32* T, u32 lo, u32 x[4], u32 k) {
  aes_round_key0(T, lo, x[0], x[1], x[2], x[3], k);
  aes_round(T, lo, x[0], x[1], x[2], x[3]);
}
__device__ __forceinline__ void echo_round(const u32* T, u32 lo, u32 W[16][4], u32 k) {
#pragma unroll
  for (int i = 0; i < 16; ++i) echo_sub(T, lo, W[i], k + (u32)i);
  echo_mix(W);
}

// kSearch: compare the top 64 bits of the X11 digest (ECHO output bytes 24..31) with
// the target and publish hits to `sink` (otedama/hitsink.h); otherwise write H.
// Round 0 only transforms the four message words (the other twelve are nonce-independent:
// x11t::ECHO_R0); in search mode round 9 only computes the two output rows the compare needs.
template <bool kSearch>
__global__ __launch_bounds__(kAesBlock) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_echo512_64(u64* __restrict__ Hb, u32 stride, u32 n, u32 base,
                                                          u64 target_hi, const HitSink sink) {
  __shared__ u32 T[kAesPrivWords];
  aes_priv_fill(T);
  const u32 lo = aes_laneoff();
  for (u32 i = blockIdx.x * kAesBlock + threadIdx.x; i < n; i += gridDim.x * kAesBlock) {
    const u32 ab = otedama_dev::abort_issue(sink);  // checked after the digest loads: one memory wait, not two
    u64 h[8];
    load_hash(Hb, stride, i, h);
    if (otedama_dev::abort_seen(ab, sink.epoch)) return;
    u32 W[16][4];
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
      for (int w = 0; w < 4; ++w) W[k][w] = x11t::ECHO_R0[k][w];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      W[8 + k][0] = lo32(h[2 * k]); W[8 + k][1] = hi32(h[2 * k]);
      W[8 + k][2] = lo32(h[2 * k + 1]); W[8 + k][3] = hi32(h[2 * k + 1]);
      echo_sub(T, lo, W[8 + k], 512u + 8u + (u32)k);
    }
    echo_mix(W);
#pragma unroll 1
    for (int r = 1; r < 9; ++r) echo_round(T, lo, W, 512u + 16u * (u32)r);
    // V' = V ^ M ^ W[0..7] ^ W[8..15]; the digest is V'[0..3], V = {512, 0, 0, 0}.
    if (kSearch) {
      // rows W'[1] (column 0: words 0, 5, 10, 15) and W'[9] (column 2: words 8, 13, 2, 7), halves 2..3
      constexpr u32 k9 = 512u + 16u * 9u;
      echo_sub(T, lo, W[0], k9 + 0); echo_sub(T, lo, W[5], k9 + 5);
      echo_sub(T, lo, W[10], k9 + 10); echo_sub(T, lo, W[15], k9 + 15);
      echo_sub(T, lo, W[8], k9 + 8); echo_sub(T, lo, W[13], k9 + 13);
      echo_sub(T, lo, W[2], k9 + 2); echo_sub(T, lo, W[7], k9 + 7);
      u32 t[2];
#pragma unroll
      for (int w = 2; w < 4; ++w) {
        const u32 r1 = xor3(xt4(W[5][w] ^ W[10][w]), W[0][w], W[10][w] ^ W[15][w]);   // column 0, row 1
        const u32 r9 = xor3(xt4(W[13][w] ^ W[2][w]), W[8][w], W[2][w] ^ W[7][w]);     // column 2, row 1
        t[w - 2] = xor3(r1, r9, w == 2 ? lo32(h[3]) : hi32(h[3]));
      }
      const u64 top = mk64(t[0], t[1]);
      if (top <= target_hi) otedama_dev::hit_publish(sink, base + i, 0u);
    } else {
      echo_round(T, lo, W, 512u + 16u * 9u);
      u64 o[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o[2 * k] = mk64(lo32(h[2 * k]) ^ W[k][0] ^ W[8 + k][0] ^ 512u, hi32(h[2 * k]) ^ W[k][1] ^ W[8 + k][1]);
        o[2 * k + 1] = mk64(lo32(h[2 * k + 1]) ^ W[k][2] ^ W[8 + k][2], hi32(h[2 * k + 1]) ^ W[k][3] ^ W[8 + k][3]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) o[4 + k] = 0;
      store_hash(Hb, stride, i, o);
    }
  }
}

}  // namespace x11k

namespace x11k {
// OTEDAMA_X11_MIDPOLL=0: the stages after BLAKE get no abort word (the A/B baseline for the cost of their polls:
// same code, a uniform kernel-argument branch instead of the load).
bool x11_midstage_polls() {
  static const bool on = [] {
    const char* v = std::getenv("OTEDAMA_X11_MIDPOLL");
    return !(v && v[0] == '0');
  }();
  return on;
}

int x11_device_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    cache[dev] = cus;
  }
  return cache[dev];
}
}  // namespace x11k

hipError_t x11_launch_stage_b(int stage, const X11Params& p, uint32_t base, uint64_t* H, uint32_t stride, uint32_t n,
                              const HitSink* sink, hipStream_t s) {
  using namespace x11k;
  const dim3 grid((n + kBlock - 1) / kBlock), block(kBlock);
  // bank-private AES table (64 KiB): 2 resident blocks of 512 per CU, grid-stride over the batch
  const u32 aes_want = (n + kAesBlock - 1) / kAesBlock, aes_cap = (u32)x11_device_cus() * 2 * 4;
  const dim3 aes_grid(aes_want < aes_cap ? aes_want : aes_cap), aes_block(kAesBlock);
  const X11Abort mid = sink && x11_midstage_polls() ? X11Abort{sink->abort, sink->epoch} : X11Abort{};
  switch (stage) {
    case kX11Shavite: k_shavite512_64<<<aes_grid, aes_block, 0, s>>>(H, stride, n, mid); break;
    case kX11Simd: {
      const dim3 g8((8ull * n + kBlock - 1) / kBlock);
      k_simd512_64<<<g8, block, 0, s>>>(H, stride, n, mid);
      break;
    }
    case kX11Echo:
      if (sink) k_echo512_64<true><<<aes_grid, aes_block, 0, s>>>(H, stride, n, base, p.target_hi, *sink);
      else k_echo512_64<false><<<aes_grid, aes_block, 0, s>>>(H, stride, n, base, p.target_hi, HitSink{});
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t x11_launch_stage(int stage, const X11Params& p, uint32_t base, uint64_t* H, uint32_t stride, uint32_t n,
                            const HitSink* sink, hipStream_t s) {
  if (stage < 0 || stage >= kX11Stages || n == 0 || stride < n || !H) return hipErrorInvalidValue;
  if (stage <= kX11Cubehash) return x11_launch_stage_a(stage, p, base, H, stride, n,
                                                       sink ? X11Abort{sink->abort, sink->epoch} : X11Abort{}, s);
  return x11_launch_stage_b(stage, p, base, H, stride, n, sink, s);
}

// The whole chain over nonces base .. base + n - 1. H: 8 * stride u64 (stride >= n).
// sink != null: search mode (ECHO compares, H keeps the SIMD output); else H = digests.
hipError_t x11_launch_chain(const X11Params& p, uint32_t base, uint64_t* H, uint32_t stride, uint32_t n,
                            const HitSink* sink, hipStream_t s) {
  // One launch per stage. Fusing the register-only middle (Skein..CubeHash) into one kernel measured
  // 1.3% slower than separate launches (its register union drops it to 4 waves/SIMD; the HBM round
  // trips it saves are hidden behind the VALU-bound stages anyway): profiles/r1/x11/NOTES.md.
  hipError_t e = hipSuccess;
  for (int st = kX11Blake; e == hipSuccess && st <= kX11Echo; ++st) e = x11_launch_stage(st, p, base, H, stride, n, sink, s);
  return e;
}

}  // namespace otedama
