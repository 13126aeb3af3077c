// CDNA4 (gfx950) integer/bitwise building blocks shared by the hash kernels.
//
// gfx950 has v_bitop3_b32 (any 3-input boolean function in one VALU op) but
// hipcc (ROCm 7.2) declines it for xor3 and splits Ch/Maj into and/or/add
// chains (measured on sha256d_search's .s: 3247 -> 2501 VALU per nonce when
// issued directly), so the boolean functions are written as inline asm.
// Truth-table immediates use the src0=0xF0, src1=0xCC, src2=0xAA convention.
// The asm statements are pure register ops (no memory, no hazards), so the
// compiler still schedules, CSEs and hoists them. Compile-time-constant inputs
// take the plain C path (`lane_varying = false`) so they constant-fold.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace otedama_dev {

__device__ __forceinline__ uint32_t ror(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t rol(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }

// `lane_varying` is a compile-time constant once the round loops unroll, so
// the untaken branch folds away.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c, bool lane_varying = true) {
  if (lane_varying) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
  }
  return a ^ b ^ c;
}
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {  // (e&f)|(~e&g)
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r) : "v"(e), "v"(f), "v"(g));
  return r;
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe8" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// SHA-256 round functions.
__device__ __forceinline__ uint32_t bS0(uint32_t a) { return xor3(ror(a, 2), ror(a, 13), ror(a, 22)); }
__device__ __forceinline__ uint32_t bS1(uint32_t e) { return xor3(ror(e, 6), ror(e, 11), ror(e, 25)); }
__device__ __forceinline__ uint32_t ss0(uint32_t x, bool v = true) { return xor3(ror(x, 7), ror(x, 18), x >> 3, v); }
__device__ __forceinline__ uint32_t ss1(uint32_t x, bool v = true) { return xor3(ror(x, 17), ror(x, 19), x >> 10, v); }

__device__ __forceinline__ constexpr uint32_t sha256_k(int i) {
  constexpr uint32_t k[64] = {
      0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
      0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
      0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
      0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
      0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
      0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
      0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
      0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
  return k[i];
}

constexpr uint32_t kSha256IVd[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

// Generic SHA-256 compression of 16 big-endian message words into st[8].
__device__ __forceinline__ void sha256_compress(uint32_t st[8], const uint32_t msg[16]) {
  uint32_t W[64];
#pragma unroll
  for (int i = 0; i < 16; ++i) W[i] = msg[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    if (t >= 16) W[t] = ss1(W[t - 2]) + W[t - 7] + ss0(W[t - 15]) + W[t - 16];
    const uint32_t t1 = h + bS1(e) + ch(e, f, g) + (sha256_k(t) + W[t]);
    const uint32_t t2 = bS0(a) + maj(a, b, c);
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

}  // namespace otedama_dev
