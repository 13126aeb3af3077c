// Device helpers shared by the X11 stage kernels (csrc/kernels/x11_*.hip).
//
// Data flow: one lane per nonce, one kernel per hash stage. The 64-byte
// intermediate digests live in HBM as a structure of arrays of 64-bit words
// (word w of nonce i at H[w * stride + i]) so every stage load/store is a fully
// coalesced 512-byte wave access; at 64 B per hash per stage the traffic is
// ~1% of the HBM roofline at the stages' ALU-bound rates. Splitting the chain
// lets every stage run at its own register budget / occupancy and keep its own
// LDS tables (Groestl 16 KiB, AES 4 KiB) instead of the union of all eleven.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "otedama/job.h"
#include "x11_tables.h"

namespace otedama {
namespace x11k {

typedef uint32_t u32;
typedef uint64_t u64;

constexpr int kBlock = 256;

__device__ __forceinline__ u64 rotl64(u64 x, int n) { return (x << n) | (x >> (64 - n)); }
__device__ __forceinline__ u64 rotr64(u64 x, int n) { return (x >> n) | (x << (64 - n)); }
__device__ __forceinline__ u32 rotl32(u32 x, int n) { return (x << n) | (x >> (32 - n)); }
__device__ __forceinline__ u32 bswap32(u32 x) { return __builtin_bswap32(x); }
__device__ __forceinline__ u64 bswap64(u64 x) { return __builtin_bswap64(x); }
__device__ __forceinline__ u32 lo32(u64 x) { return (u32)x; }
__device__ __forceinline__ u32 hi32(u64 x) { return (u32)(x >> 32); }
__device__ __forceinline__ u64 mk64(u32 lo, u32 hi) { return (u64)lo | ((u64)hi << 32); }

__device__ __forceinline__ void load_hash(const u64* __restrict__ H, u32 stride, u32 i, u64 h[8]) {
#pragma unroll
  for (int w = 0; w < 8; ++w) h[w] = __builtin_nontemporal_load(H + (size_t)w * stride + i);
}
__device__ __forceinline__ void store_hash(u64* __restrict__ H, u32 stride, u32 i, const u64 h[8]) {
#pragma unroll
  for (int w = 0; w < 8; ++w) __builtin_nontemporal_store(h[w], H + (size_t)w * stride + i);
}

// AES T-tables in LDS: T[r][x] = rotl32(AES_T0[x], 8r).
__device__ __forceinline__ void aes_tables_to_lds(u32 (*T)[256]) {
  for (int x = threadIdx.x; x < 256; x += blockDim.x) {
    const u32 v = x11t::AES_T0[x];
    T[0][x] = v;
    T[1][x] = rotl32(v, 8);
    T[2][x] = rotl32(v, 16);
    T[3][x] = rotl32(v, 24);
  }
  __syncthreads();
}
// Keyless AES round (SubBytes, ShiftRows, MixColumns) on four LE column words.
__device__ __forceinline__ void aes_round(const u32 (*T)[256], u32& x0, u32& x1, u32& x2, u32& x3) {
  const u32 y0 = T[0][x0 & 0xff] ^ T[1][(x1 >> 8) & 0xff] ^ T[2][(x2 >> 16) & 0xff] ^ T[3][x3 >> 24];
  const u32 y1 = T[0][x1 & 0xff] ^ T[1][(x2 >> 8) & 0xff] ^ T[2][(x3 >> 16) & 0xff] ^ T[3][x0 >> 24];
  const u32 y2 = T[0][x2 & 0xff] ^ T[1][(x3 >> 8) & 0xff] ^ T[2][(x0 >> 16) & 0xff] ^ T[3][x1 >> 24];
  const u32 y3 = T[0][x3 & 0xff] ^ T[1][(x0 >> 8) & 0xff] ^ T[2][(x1 >> 16) & 0xff] ^ T[3][x2 >> 24];
  x0 = y0; x1 = y1; x2 = y2; x3 = y3;
}

}  // namespace x11k

// Stage ids (chain order) and launchers.
enum X11Stage : int {
  kX11Blake = 0, kX11Bmw, kX11Groestl, kX11Skein, kX11Jh, kX11Keccak,
  kX11Luffa, kX11Cubehash, kX11Shavite, kX11Simd, kX11Echo, kX11Stages
};

// Stage 0 writes H from the header + nonces; stages 1..10 transform H in place.
// Stage 10 with `out` != null compares against the target and appends nonces
// instead of writing H (search mode).
hipError_t x11_launch_stage_a(int stage, const X11Params& p, uint32_t base, uint64_t* H, uint32_t stride, uint32_t n,
                              hipStream_t s);
hipError_t x11_launch_stage_b(int stage, const X11Params& p, uint32_t base, uint64_t* H, uint32_t stride, uint32_t n,
                              uint32_t* out, uint32_t cap, hipStream_t s);

}  // namespace otedama
