// Device helpers shared by the X11 stage kernels (csrc/kernels/x11_*.hip).
//
// Data flow: one lane per nonce, one kernel per hash stage. The 64-byte
// intermediate digests live in HBM as a structure of arrays of 64-bit words
// (word w of nonce i at H[w * stride + i]) so every stage load/store is a fully
// coalesced 512-byte wave access; at 64 B per hash per stage the traffic is
// ~1% of the HBM roofline at the stages' ALU-bound rates. Splitting the chain
// lets every stage run at its own register budget / occupancy and keep its own
// LDS tables (bank-private 64 KiB Groestl / AES tables) instead of the union of all eleven.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "otedama/job.h"
#include "cdna_bitops.h"
#include "hitsink_dev.h"
#include "x11_tables.h"

namespace otedama {
namespace x11k {

typedef uint32_t u32;
typedef uint64_t u64;
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));  // packed 16-bit VALU ops (v_pk_*)

constexpr int kBlock = 256;

// 64-bit rotates as two v_alignbit_b32 (hipcc otherwise emits a 64-bit shift pair + two ors).
// n is a compile-time constant once the round loops unroll, so the branches fold.
__device__ __forceinline__ u64 rotl64(u64 x, int n) {
  const u32 lo = (u32)x, hi = (u32)(x >> 32);
  if ((n & 63) == 0) return x;
  if (n == 32) return (u64)hi | ((u64)lo << 32);
  if (n < 32)
    return (u64)__builtin_amdgcn_alignbit(lo, hi, 32 - n) | ((u64)__builtin_amdgcn_alignbit(hi, lo, 32 - n) << 32);
  return (u64)__builtin_amdgcn_alignbit(hi, lo, 64 - n) | ((u64)__builtin_amdgcn_alignbit(lo, hi, 64 - n) << 32);
}
__device__ __forceinline__ u64 rotr64(u64 x, int n) { return rotl64(x, (64 - n) & 63); }
__device__ __forceinline__ u32 rotl32(u32 x, int n) { return __builtin_amdgcn_alignbit(x, x, (32 - n) & 31); }
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

// Any 3-input boolean function / xor3 in one v_bitop3_b32 (hipcc rarely forms it itself).
using otedama_dev::xor3;
template <unsigned TT>
__device__ __forceinline__ u32 bop3(u32 a, u32 b, u32 c) {
  u32 r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4" : "=v"(r) : "v"(a), "v"(b), "v"(c), "i"(TT));
  return r;
}
__device__ __forceinline__ u64 xor3_64(u64 a, u64 b, u64 c) { return mk64(xor3(lo32(a), lo32(b), lo32(c)), xor3(hi32(a), hi32(b), hi32(c))); }

// ---------------------------------------------------------------- bank-private tables
// Random 8-bit table lookups from a shared table cost ~3.1x their conflict-free LDS time on
// gfx950 (measured: SQ_LDS_BANK_CONFLICT = 67% of SQ_LDS_IDX_ACTIVE for Groestl/ECHO/SHAvite,
// profiles/r1/x11/pmc_baseline.csv). Here every lane reads its own copy of the table, placed so
// that lane l only ever touches bank(s) owned by l inside its 32-lane half-wave: conflict-free.
// The address of entry x is (x << 8) | lane_offset, built with one v_perm_b32 straight from the
// state word (byte k of w -> address byte 1, lane offset -> byte 0).
__device__ __forceinline__ u32 lds_addr(u32 w, int k, u32 laneoff) {
  return __builtin_amdgcn_perm(w, laneoff, 0x0c0c0000u | ((4u + (u32)k) << 8));
}

// AES: T0 and T1 = rotl8(T0) (T2, T3 are their rotl16), 32 copies each in one 64 KiB image: the 256-byte row
// of entry x holds T0[x] for lanes l mod 32 in bytes 0..127 and T1[x] in bytes 128..255. ds_read_b32 serves lanes
// {0-31} and {32-63} in separate LDS cycles with bank (a/4) mod 32, so lane l -> bank l mod 32 for either table:
// conflict-free. A column is T0[b0] ^ T1[b1] ^ rotl16(T0[b2] ^ T1[b3]): one rotate instead of three.
constexpr u32 kAesPrivWords = 256 * 64;
__device__ __forceinline__ void aes_priv_fill(u32* T) {
  for (u32 c = threadIdx.x; c < kAesPrivWords / 4; c += blockDim.x) {
    const u32 t0 = x11t::AES_T0[c >> 4];
    const u32 v = (c & 15u) < 8u ? t0 : rotl32(t0, 8);
    reinterpret_cast<uint4*>(T)[c] = make_uint4(v, v, v, v);
  }
  __syncthreads();
}
__device__ __forceinline__ u32 aes_laneoff() { return (threadIdx.x & 31u) << 2; }
__device__ __forceinline__ u32 aes_lk(const u32* T, u32 lo, u32 w, int k) {
  return *reinterpret_cast<const u32*>(reinterpret_cast<const char*>(T) + lds_addr(w, k, lo));
}
// AES round (SubBytes, ShiftRows, MixColumns) on four LE column words, then AddRoundKey.
#define AES_COLS_(T, lo, x0, x1, x2, x3)                                                                   \
  const u32 lo1_ = (lo) | 0x80u;                                                                        \
  const u32 a0 = aes_lk(T, lo, x0, 0), a1 = aes_lk(T, lo1_, x1, 1), a2 = aes_lk(T, lo, x2, 2),        \
            a3 = aes_lk(T, lo1_, x3, 3);                                                              \
  const u32 b0 = aes_lk(T, lo, x1, 0), b1 = aes_lk(T, lo1_, x2, 1), b2 = aes_lk(T, lo, x3, 2),        \
            b3 = aes_lk(T, lo1_, x0, 3);                                                              \
  const u32 c0 = aes_lk(T, lo, x2, 0), c1 = aes_lk(T, lo1_, x3, 1), c2 = aes_lk(T, lo, x0, 2),        \
            c3 = aes_lk(T, lo1_, x1, 3);                                                              \
  const u32 d0 = aes_lk(T, lo, x3, 0), d1 = aes_lk(T, lo1_, x0, 1), d2 = aes_lk(T, lo, x1, 2),        \
            d3 = aes_lk(T, lo1_, x2, 3)
__device__ __forceinline__ void aes_round_k(const u32* T, u32 lo, u32& x0, u32& x1, u32& x2, u32& x3, u32 k0, u32 k1,
                                            u32 k2, u32 k3) {
  AES_COLS_(T, lo, x0, x1, x2, x3);
  x0 = xor3(a0, a1, k0) ^ rotl32(a2 ^ a3, 16);
  x1 = xor3(b0, b1, k1) ^ rotl32(b2 ^ b3, 16);
  x2 = xor3(c0, c1, k2) ^ rotl32(c2 ^ c3, 16);
  x3 = xor3(d0, d1, k3) ^ rotl32(d2 ^ d3, 16);
}
// k0 is ECHO's wave-uniform counter key.
__device__ __forceinline__ void aes_round_key0(const u32* T, u32 lo, u32& x0, u32& x1, u32& x2, u32& x3, u32 k0) {
  AES_COLS_(T, lo, x0, x1, x2, x3);
  x0 = xor3(a0, a1, rotl32(a2 ^ a3, 16)) ^ k0;
  x1 = xor3(b0, b1, rotl32(b2 ^ b3, 16));
  x2 = xor3(c0, c1, rotl32(c2 ^ c3, 16));
  x3 = xor3(d0, d1, rotl32(d2 ^ d3, 16));
}
__device__ __forceinline__ void aes_round(const u32* T, u32 lo, u32& x0, u32& x1, u32& x2, u32& x3) {
  AES_COLS_(T, lo, x0, x1, x2, x3);
  x0 = xor3(a0, a1, rotl32(a2 ^ a3, 16));
  x1 = xor3(b0, b1, rotl32(b2 ^ b3, 16));
  x2 = xor3(c0, c1, rotl32(c2 ^ c3, 16));
  x3 = xor3(d0, d1, rotl32(d2 ^ d3, 16));
}
#undef AES_COLS_

// Groestl: T0 only (row r is rotl64(T0, 8r); rows r and r+4 differ by a half swap, which is free),
// 32 copies, qword 32x + (l mod 32) = T0[x] (ds_read_b64 banks are (a/4) mod 64 per 32-lane half:
// lane l -> banks 2l, 2l+1). 64 KiB.
constexpr u32 kGroestlPrivQwords = 256 * 32;
__device__ __forceinline__ void groestl_priv_fill(u64* T) {
  for (u32 c = threadIdx.x; c < kGroestlPrivQwords / 2; c += blockDim.x) {
    const u64 v = x11t::GROESTL_T0[c >> 4];
    reinterpret_cast<uint4*>(T)[c] = make_uint4(lo32(v), hi32(v), lo32(v), hi32(v));
  }
  __syncthreads();
}
__device__ __forceinline__ u32 groestl_laneoff() { return (threadIdx.x & 31u) << 3; }
__device__ __forceinline__ u64 groestl_lk(const u64* T, u32 lo, u32 w, int k) {
  return *reinterpret_cast<const u64*>(reinterpret_cast<const char*>(T) + lds_addr(w, k, lo));
}

// Grid for a grid-stride kernel: enough resident blocks to fill every CU `per_cu` times over.
int x11_device_cus();
bool x11_midstage_polls();  // stages after BLAKE poll the abort word (OTEDAMA_X11_MIDPOLL=0 turns it off)

}  // namespace x11k

// Stage ids (chain order) and launchers.
enum X11Stage : int {
  kX11Blake = 0, kX11Bmw, kX11Groestl, kX11Skein, kX11Jh, kX11Keccak,
  kX11Luffa, kX11Cubehash, kX11Shavite, kX11Simd, kX11Echo, kX11Stages
};

// Stage 0 writes H from the header + nonces; stages 1..10 transform H in place.
// Stage 10 with `out` != null compares against the target and appends nonces
// instead of writing H (search mode).
// Abort word of the batch (otedama/hitsink.h), polled by every stage once the host moved it past `epoch`
// (word == nullptr: never). BLAKE checks before hashing; each later stage issues the load before its digest load and
// tests it after (x11_abort_issue / x11_abort_seen), so the poll's latency hides under the digest read instead of
// stalling the wave (round 3's stall-on-load polls cost 1-7% per stage, profiles/r3/f_regressions). A superseded
// batch then stops at the next stage boundary instead of running its remaining stages (~18 ms at 2^23 nonces).
struct X11Abort {
  const uint32_t* word = nullptr;
  uint32_t epoch = 0;
};
__device__ __forceinline__ bool x11_stop(const X11Abort& a) {
  return otedama_dev::abort_newer(otedama_dev::abort_peek(a.word, a.epoch), a.epoch);
}
__device__ __forceinline__ uint32_t x11_abort_issue(const X11Abort& a) {
  if (a.word == nullptr) return a.epoch;
  return __hip_atomic_load(const_cast<uint32_t*>(a.word), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool x11_abort_seen(uint32_t raw, const X11Abort& a) {
  return otedama_dev::abort_seen(raw, a.epoch);
}
hipError_t x11_launch_stage_a(int stage, const X11Params& p, uint32_t base, uint64_t* H, uint32_t stride, uint32_t n,
                              X11Abort ab, hipStream_t s);
// sink == nullptr: ECHO writes the digests (trace mode); else it compares and publishes hits to *sink.
hipError_t x11_launch_stage_b(int stage, const X11Params& p, uint32_t base, uint64_t* H, uint32_t stride, uint32_t n,
                              const HitSink* sink, hipStream_t s);

}  // namespace otedama
