// scrypt_search — Litecoin-parameter scrypt (N=1024, r=1, p=1) nonce search on
// gfx950. [NO REFERENCE CODE]: v3 of the reference removed scrypt PoW
// (CHANGELOG.md:6623); the only scrypt there is the wallet KDF
// (internal/lightning/seedstore.go:68-72). BASELINE.json config 3.
//
// Design: one lane = one hash. The 128 KiB ROMix scratchpad of
// every in-flight lane lives in HBM (hundreds of thousands of lanes = tens of GB,
// sized against the 288 GB of HBM3E), laid out wave-blocked:
//     V[wave][i / GAP][lane]   (one 128-byte entry = 8 x uint4)
// so the write phase is a fully coalesced 8 KiB store per wave per entry, a
// read-phase lookup is one full 128-byte line per lane, and each wave's lookups
// stay inside its own contiguous 8 MiB region (TLB reach). GAP > 1 is the
// lookup-gap time/memory trade-off: only every GAP-th entry is stored and the
// missing ones are recomputed from the previous stored entry.
// PBKDF2-HMAC-SHA256 runs per lane (the HMAC key is the header, which holds the
// nonce); only SHA-256 of header bytes 0..63 is hoisted to the host.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cdna_bitops.h"
#include "hitsink_dev.h"
#include <cstdlib>
#include <cstring>

#include "otedama/job.h"

namespace {

using namespace otedama_dev;

__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ void salsa20_8(uint32_t B[16]) {
  uint32_t x0 = B[0], x1 = B[1], x2 = B[2], x3 = B[3], x4 = B[4], x5 = B[5], x6 = B[6], x7 = B[7];
  uint32_t x8 = B[8], x9 = B[9], x10 = B[10], x11 = B[11], x12 = B[12], x13 = B[13], x14 = B[14], x15 = B[15];
#pragma unroll
  for (int i = 0; i < 8; i += 2) {
    x4 ^= rol(x0 + x12, 7);   x8 ^= rol(x4 + x0, 9);    x12 ^= rol(x8 + x4, 13);   x0 ^= rol(x12 + x8, 18);
    x9 ^= rol(x5 + x1, 7);    x13 ^= rol(x9 + x5, 9);   x1 ^= rol(x13 + x9, 13);   x5 ^= rol(x1 + x13, 18);
    x14 ^= rol(x10 + x6, 7);  x2 ^= rol(x14 + x10, 9);  x6 ^= rol(x2 + x14, 13);   x10 ^= rol(x6 + x2, 18);
    x3 ^= rol(x15 + x11, 7);  x7 ^= rol(x3 + x15, 9);   x11 ^= rol(x7 + x3, 13);   x15 ^= rol(x11 + x7, 18);
    x1 ^= rol(x0 + x3, 7);    x2 ^= rol(x1 + x0, 9);    x3 ^= rol(x2 + x1, 13);    x0 ^= rol(x3 + x2, 18);
    x6 ^= rol(x5 + x4, 7);    x7 ^= rol(x6 + x5, 9);    x4 ^= rol(x7 + x6, 13);    x5 ^= rol(x4 + x7, 18);
    x11 ^= rol(x10 + x9, 7);  x8 ^= rol(x11 + x10, 9);  x9 ^= rol(x8 + x11, 13);   x10 ^= rol(x9 + x8, 18);
    x12 ^= rol(x15 + x14, 7); x13 ^= rol(x12 + x15, 9); x14 ^= rol(x13 + x12, 13); x15 ^= rol(x14 + x13, 18);
  }
  B[0] += x0; B[1] += x1; B[2] += x2; B[3] += x3; B[4] += x4; B[5] += x5; B[6] += x6; B[7] += x7;
  B[8] += x8; B[9] += x9; B[10] += x10; B[11] += x11; B[12] += x12; B[13] += x13; B[14] += x14; B[15] += x15;
}

// BlockMix_salsa20/8 with r = 1: X = [B0 | B1] (32 words).
__device__ __forceinline__ void blockmix(uint32_t X[32]) {
#pragma unroll
  for (int k = 0; k < 16; ++k) X[k] ^= X[16 + k];
  salsa20_8(X);
#pragma unroll
  for (int k = 0; k < 16; ++k) X[16 + k] ^= X[k];
  salsa20_8(X + 16);
}

__device__ __forceinline__ void store_entry(uint4* __restrict__ dst, const uint32_t X[32]) {
#pragma unroll
  for (int q = 0; q < 8; ++q) dst[q] = make_uint4(X[4 * q], X[4 * q + 1], X[4 * q + 2], X[4 * q + 3]);
}
__device__ __forceinline__ void load_entry(const uint4* __restrict__ src, uint32_t T[32]) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint4 v = src[q];
    T[4 * q] = v.x; T[4 * q + 1] = v.y; T[4 * q + 2] = v.z; T[4 * q + 3] = v.w;
  }
}

// HMAC-SHA256 pad states for key K' (8 words).
__device__ __forceinline__ void hmac_states(const uint32_t key[8], uint32_t istate[8], uint32_t ostate[8]) {
  uint32_t blk[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) blk[i] = key[i] ^ 0x36363636u;
#pragma unroll
  for (int i = 8; i < 16; ++i) blk[i] = 0x36363636u;
#pragma unroll
  for (int i = 0; i < 8; ++i) istate[i] = kSha256IVd[i];
  sha256_compress(istate, blk);
#pragma unroll
  for (int i = 0; i < 8; ++i) blk[i] = key[i] ^ 0x5c5c5c5cu;
#pragma unroll
  for (int i = 8; i < 16; ++i) blk[i] = 0x5c5c5c5cu;
#pragma unroll
  for (int i = 0; i < 8; ++i) ostate[i] = kSha256IVd[i];
  sha256_compress(ostate, blk);
}

// Outer HMAC step: H(opad-state || digest) with fixed padding (768-bit message).
__device__ __forceinline__ void hmac_outer(const uint32_t ostate[8], const uint32_t digest[8], uint32_t out[8]) {
  uint32_t blk[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) blk[i] = digest[i];
  blk[8] = 0x80000000u;
#pragma unroll
  for (int i = 9; i < 15; ++i) blk[i] = 0u;
  blk[15] = 768u;
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = ostate[i];
  sha256_compress(out, blk);
}

// Stage 1: PBKDF2 #1 for `nonce` -> X[32] (LE words of the 128-byte B).
__device__ __forceinline__ void scrypt_pbkdf_in(const otedama::ScryptParams& p, uint32_t nonce, uint32_t X[32]) {
  // K' = SHA-256(header80) (key longer than the block size).
  uint32_t hdrbe[20];
#pragma unroll
  for (int i = 0; i < 19; ++i) hdrbe[i] = bswap(p.hdr[i]);
  hdrbe[19] = bswap(nonce);
  uint32_t key[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) key[i] = p.hmid[i];
  {
    uint32_t blk[16] = {hdrbe[16], hdrbe[17], hdrbe[18], hdrbe[19], 0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 640u};
    sha256_compress(key, blk);
  }
  uint32_t istate[8], ostate[8];
  hmac_states(key, istate, ostate);
  // salt = header80, 4 blocks of 32 bytes.
  uint32_t ist2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) ist2[i] = istate[i];
  sha256_compress(ist2, hdrbe);  // header bytes 0..63
#pragma unroll
  for (int blkno = 1; blkno <= 4; ++blkno) {
    uint32_t st[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = ist2[i];
    uint32_t blk[16] = {hdrbe[16], hdrbe[17], hdrbe[18], hdrbe[19], uint32_t(blkno), 0x80000000u,
                        0, 0, 0, 0, 0, 0, 0, 0, 0, (64u + 84u) * 8u};
    sha256_compress(st, blk);
    uint32_t t[8];
    hmac_outer(ostate, st, t);
#pragma unroll
    for (int i = 0; i < 8; ++i) X[8 * (blkno - 1) + i] = bswap(t[i]);
  }
}

// Stage 3: PBKDF2 #2 over X (salt = X || INT(1)); returns final state word 7.
__device__ __forceinline__ uint32_t scrypt_pbkdf_out(const otedama::ScryptParams& p, uint32_t nonce,
                                                     const uint32_t X[32]) {
  uint32_t key[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) key[i] = p.hmid[i];
  {
    uint32_t blk[16] = {bswap(p.hdr[16]), bswap(p.hdr[17]), bswap(p.hdr[18]), bswap(nonce), 0x80000000u,
                        0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 640u};
    sha256_compress(key, blk);
  }
  uint32_t istate[8], ostate[8];
  hmac_states(key, istate, ostate);
  uint32_t st[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) st[i] = istate[i];
  uint32_t blk[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) blk[i] = bswap(X[i]);
  sha256_compress(st, blk);
#pragma unroll
  for (int i = 0; i < 16; ++i) blk[i] = bswap(X[16 + i]);
  sha256_compress(st, blk);
  uint32_t tail[16] = {1u, 0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, (64u + 132u) * 8u};
  sha256_compress(st, tail);
  uint32_t out[8];
  hmac_outer(ostate, st, out);
  return out[7];
}

// Stage 2: ROMix on X in place. `Vw` is this wave's scratch region: entry e of
// lane l at Vw[(e * 64 + l) * 8] (uint4 units). A wave's region is contiguous
// (64 lanes x 1024/GAP entries x 128 B = 8 MiB at GAP 1), so write-phase
// stores are 8 KiB-contiguous per wave and read-phase lookups stay inside a few
// large pages; an entry-major layout over the whole (tens of GB) pad measured
// 7.7 MH/s and got slower as lanes grew (TLB reach), see profiles/.
template <int GAP>
__device__ __forceinline__ void scrypt_romix(uint32_t X[32], uint4* __restrict__ Vw, uint32_t lane) {
  for (int i = 0; i < 1024; ++i) {
    if (i % GAP == 0) store_entry(Vw + ((uint64_t(i / GAP) * 64u + lane) << 3), X);
    blockmix(X);
  }
  for (int i = 0; i < 1024; ++i) {
    const uint32_t j = X[16] & 1023u;
    uint32_t T[32];
    load_entry(Vw + ((uint64_t(j / GAP) * 64u + lane) << 3), T);
    if constexpr (GAP > 1) {
      for (uint32_t r = 0; r < (j % GAP); ++r) blockmix(T);
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) X[k] ^= T[k];
    blockmix(X);
  }
}

// ---------------------------------------------------------------------------
// Lane-cooperative ROMix (GAP 1). Measured on the per-lane kernel above
// (profiles/r1): the texture path is ~95% busy and L2 sees ~3 read requests per
// 128-byte lookup, because every vector-memory instruction carries 64 lanes x
// 16 B of 64 unrelated lines - the 8 partial-line loads of an entry thrash the
// L1 between instructions, and the 8 partial-line stores of the write phase
// cost the same address/tag work. Here every pad access is full-line: the 8
// lanes of an octet move ONE 128-byte entry (lane `slot` handles chunk
// slot ^ swz(owner)), and entries change hands through a wave-private 4 KiB LDS
// tile (32 owner rows of 8 chunks; owner s's chunk c at s*8 + (c ^ swz(s)), so
// owner-side ds_*_b128 and the lane-linear octet side are both conflict-free).
//   write phase: owners stage X into the tile, octets store full lines (2 halves)
//   read phase : owners 0..31 by LDS-DMA (buffer_load ... lds), owners 32..63
//                register-staged, ONE vmcnt wait per lookup, then the staged
//                half is written to the tile after the first half is consumed.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void glds_lptr_t;
typedef unsigned coop_v4u __attribute__((ext_vector_type(4)));

// Pad stores are streaming (nt): the write phase is store-only traffic that is read back at most once,
// much later. tools/bench_hbm.hip: sequential full-line stores 3.3 TB/s plain vs 5.8 TB/s nt.
#ifndef OTD_SCRYPT_STORE_CPOL
#define OTD_SCRYPT_STORE_CPOL 2  // gfx950 cache policy bits: 1 = sc0, 2 = nt, 16 = sc1
#endif
constexpr int kStoreNT = OTD_SCRYPT_STORE_CPOL;

__device__ __forceinline__ uint32_t coop_swz(uint32_t s_local) {
  return ((s_local >> 1) & 3u) | (((s_local >> 3) & 1u) << 2);
}

// tile: this wave's 4 KiB LDS tile (wave-uniform). rs: buffer descriptor over this wave's 8 MiB pad.
// LCPOL: cache policy of the lookup loads (0 = default, 2 = nt).
// Cooperative store of pad entry i (X of all 64 lanes) as 64 full-line nt stores (two halves through the tile).
__device__ __forceinline__ void coop_store_entry(const uint32_t X[32], __amdgpu_buffer_rsrc_t rs, uint4* __restrict__ tile,
                                                 uint32_t lane, uint32_t i) {
  char* tb = reinterpret_cast<char*>(tile);
  // Lane-derived constants are recomputed per call (a few VALU) rather than hoisted into loop-invariant
  // VGPRs that would stay live through BlockMix and cost occupancy.
  uint32_t ln = lane;
  asm volatile("" : "+v"(ln));
  const uint32_t slot = ln & 7u, octet = ln >> 3, own = ln & 31u;
  const uint32_t rd = (own << 7) ^ (coop_swz(own) << 4);  // owner row, swizzled chunk 0 (bytes)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // previous reads of the tile retired
    if ((ln >> 5) == uint32_t(h)) {
#pragma unroll
      for (int c = 0; c < 8; ++c)
        *reinterpret_cast<uint4*>(tb + (rd ^ (uint32_t(c) << 4))) =
            make_uint4(X[4 * c], X[4 * c + 1], X[4 * c + 2], X[4 * c + 3]);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint4 v = tile[64 * r + ln];
      const uint32_t owner = uint32_t(32 * h + 8 * r) + octet;
      const uint32_t chunk = slot ^ (((octet >> 1) & 3u) | (uint32_t(r & 1) << 2));  // slot ^ swz(8r+octet)
      const coop_v4u vv = {v.x, v.y, v.z, v.w};
      __builtin_amdgcn_raw_buffer_store_b128(vv, rs, (i << 13) | (owner << 7) | (chunk << 4), 0, kStoreNT);
    }
  }
}

// Issue the cooperative lookup V[X[16] & 1023] for all 64 lanes: owners 0..31 by LDS-DMA into the tile,
// owners 32..63 into R (register staging). Completed by coop_consume.
template <int LCPOL>
__device__ __forceinline__ void coop_issue(const uint32_t X[32], __amdgpu_buffer_rsrc_t rs, uint4* __restrict__ tile,
                                           uint32_t lane, coop_v4u R[4]) {
  uint32_t ln = lane;
  asm volatile("" : "+v"(ln));
  const uint32_t slot = ln & 7u, octet = ln >> 3;
  const uint32_t j = X[16] & 1023u;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // tile free (previous consumer's reads retired)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t chunk = slot ^ (((octet >> 1) & 3u) | (uint32_t(r & 1) << 2));
    const uint32_t o0 = uint32_t(8 * r) + octet, o1 = o0 + 32u;
    const uint32_t j0 = uint32_t(__shfl(int(j), int(o0), 64));
    const uint32_t j1 = uint32_t(__shfl(int(j), int(o1), 64));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (glds_lptr_t*)(tile + 64 * r), 16, (j0 << 13) | (o0 << 7) | (chunk << 4),
                                             0, 0, LCPOL);
    R[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, (j1 << 13) | (o1 << 7) | (chunk << 4), 0, LCPOL);
  }
}

// X ^= the looked-up entry (one vmcnt wait; the register-staged half goes through the tile second).
__device__ __forceinline__ void coop_consume(uint32_t X[32], uint4* __restrict__ tile, uint32_t lane,
                                             const coop_v4u R[4]) {
  const char* tb = reinterpret_cast<const char*>(tile);
  uint32_t ln = lane;
  asm volatile("" : "+v"(ln));
  const uint32_t own = ln & 31u;
  const uint32_t rd = (own << 7) ^ (coop_swz(own) << 4);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (ln < 32u) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const uint4 t = *reinterpret_cast<const uint4*>(tb + (rd ^ (uint32_t(c) << 4)));
      X[4 * c] ^= t.x; X[4 * c + 1] ^= t.y; X[4 * c + 2] ^= t.z; X[4 * c + 3] ^= t.w;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int r = 0; r < 4; ++r) tile[64 * r + ln] = make_uint4(R[r].x, R[r].y, R[r].z, R[r].w);
  __builtin_amdgcn_wave_barrier();
  if (ln >= 32u) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const uint4 t = *reinterpret_cast<const uint4*>(tb + (rd ^ (uint32_t(c) << 4)));
      X[4 * c] ^= t.x; X[4 * c + 1] ^= t.y; X[4 * c + 2] ^= t.z; X[4 * c + 3] ^= t.w;
    }
  }
}

// The abort word (otedama/hitsink.h) is polled before each ROMix phase (a wave's hash takes ~32 ms, its phases
// ~16 ms each), and every POLL iterations of the write phase by the scalar unit. A vector poll inside the BlockMix
// loops made the allocator reload spilled values every iteration (64-VGPR budget), and splitting each loop in two
// cost 0.9% of ROMix time (four loop bodies in the instruction cache, profiles/r3/f_regressions). The scalar poll
// between chunks of the write loop keeps that loop's body and allocation (+1 instruction per iteration, no new
// spill); in the read loop the same structure cost 2 scratch reloads and ~30 instructions per iteration, so the read
// phase keeps only its boundary poll. The miner runs its two batches half a hash apart (gpu_miner.hip), so one of
// them is always in its write phase and stops within ~1 ms of new work. POLL = 1024: boundary polls only.
// Returns false when aborted.
template <int LCPOL, int POLL>
__device__ __forceinline__ bool scrypt_romix_coop(uint32_t X[32], __amdgpu_buffer_rsrc_t rs, uint4* __restrict__ tile,
                                                  uint32_t lane, const otedama::HitSink& sink) {
  static_assert(POLL > 0 && 1024 % POLL == 0, "poll interval must divide the ROMix loop");
  if (abort_newer(abort_peek(sink), sink.epoch)) return false;
  // chunks of POLL iterations, the scalar poll (no VGPR) between them: an exit edge inside the loop itself cost 10
  // more spilled VGPRs
  for (uint32_t c = 0; c < 1024; c += POLL) {
    if (c && abort_newer(abort_peek_scalar(sink), sink.epoch)) return false;
    for (uint32_t i = c; i < c + POLL; ++i) {
      coop_store_entry(X, rs, tile, lane, i);
      blockmix(X);
    }
  }
  if (abort_newer(abort_peek(sink), sink.epoch)) return false;
  for (int i = 0; i < 1024; ++i) {
    coop_v4u R[4];
    coop_issue<LCPOL>(X, rs, tile, lane, R);
    coop_consume(X, tile, lane, R);
    blockmix(X);
  }
  return true;
}

// The two ROMix phases as separate launches (see otd_scrypt_romix_coop_phase): PHASE 1 writes the pad, PHASE 2
// does the 1024 lookups. X crosses the launch boundary through xbuf and the pad stays in HBM.
template <int LCPOL, int PHASE>
__device__ __forceinline__ void scrypt_romix_coop_phase(uint32_t X[32], __amdgpu_buffer_rsrc_t rs,
                                                        uint4* __restrict__ tile, uint32_t lane) {
  if constexpr (PHASE == 1) {
    for (uint32_t i = 0; i < 1024; ++i) {
      coop_store_entry(X, rs, tile, lane, i);
      blockmix(X);
    }
  } else {
    for (int i = 0; i < 1024; ++i) {
      coop_v4u R[4];
      coop_issue<LCPOL>(X, rs, tile, lane, R);
      coop_consume(X, tile, lane, R);
      blockmix(X);
    }
  }
}

// Two hashes per lane (A, B), software-pipelined so each stream's BlockMix runs while the other stream's
// lookup is in flight; the wave only waits when a lookup outlives a whole BlockMix. One tile and one R are
// shared: at most one lookup is outstanding per wave at any time.
template <int LCPOL>
__device__ __forceinline__ void scrypt_romix_coop2(uint32_t XA[32], uint32_t XB[32], __amdgpu_buffer_rsrc_t rsA,
                                                   __amdgpu_buffer_rsrc_t rsB, uint4* __restrict__ tile, uint32_t lane) {
  for (uint32_t i = 0; i < 1024; ++i) {
    coop_store_entry(XA, rsA, tile, lane, i);
    blockmix(XA);
    coop_store_entry(XB, rsB, tile, lane, i);
    blockmix(XB);
  }
  coop_v4u R[4];
  coop_issue<LCPOL>(XA, rsA, tile, lane, R);
  for (int i = 0; i < 1024; ++i) {
    coop_consume(XA, tile, lane, R);
    coop_issue<LCPOL>(XB, rsB, tile, lane, R);
    blockmix(XA);
    coop_consume(XB, tile, lane, R);
    if (i < 1023) coop_issue<LCPOL>(XA, rsA, tile, lane, R);
    blockmix(XB);
  }
}

}  // namespace

// The three stages are separate launches so the ROMix kernel is register-lean
// (X, T and the salsa state only): fused, the unrolled SHA-256 schedules of the
// PBKDF2 layers pushed the kernel to 256 VGPRs (1-2 waves/SIMD). The stages
// exchange 128 bytes per hash through `xbuf` (0.1% of the ROMix traffic).
extern "C" __global__ __launch_bounds__(256) void otd_scrypt_pbkdf_in(const otedama::ScryptParams p, uint32_t base,
                                                                      uint32_t count, uint4* __restrict__ xbuf) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  uint32_t X[32];
  scrypt_pbkdf_in(p, base + i, X);
  store_entry(xbuf + (uint64_t(i) << 3), X);
}

template <int GAP>
__global__ __launch_bounds__(256) void otd_scrypt_romix(uint32_t count, uint4* __restrict__ xbuf,
                                                        uint4* __restrict__ V) {
  const uint64_t slot = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t nslots = uint64_t(gridDim.x) * blockDim.x;
  uint4* Vw = V + (slot >> 6) * (uint64_t(1024 / GAP) * 64u * 8u);
  const uint32_t lane = uint32_t(slot & 63u);
  for (uint64_t i = slot; i < count; i += nslots) {
    uint32_t X[32];
    load_entry(xbuf + (i << 3), X);
    scrypt_romix<GAP>(X, Vw, lane);
    store_entry(xbuf + (i << 3), X);
  }
}

template <int LCPOL, int POLL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void otd_scrypt_romix_coop(uint32_t count, uint4* __restrict__ xbuf,
                                                             uint4* __restrict__ V, const otedama::HitSink sink) {
  __shared__ uint4 tiles[4 * 256];  // 4 waves x 4 KiB half-tiles
  const uint64_t slot = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t nslots = uint64_t(gridDim.x) * blockDim.x;
  const uint32_t lane = uint32_t(slot & 63u);
  // Wave-uniform values made provably uniform (readfirstlane) so the pad descriptor and the LDS-DMA base
  // (M0) live in SGPRs.
  const uint64_t wave = (uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(slot >> 32))) << 26) |
                        uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(slot) >> 6));
  uint4* Vw = V + wave * (1024ull * 64u * 8u);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(Vw, (short)0, 1024 * 64 * 128, 0x00020000);
  (void)Vw;
  uint4* tile = tiles + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * 256;
  // count is a multiple of 64 (launcher rounds up), so whole waves iterate together and every lane of a wave
  // reaches the cooperative loads and __shfl.
  for (uint64_t i = slot; i < count; i += nslots) {
    uint32_t X[32];
    load_entry(xbuf + (i << 3), X);
    if (!scrypt_romix_coop<LCPOL, POLL>(X, rs, tile, lane, sink)) return;  // aborted: pbkdf_out publishes nothing
    store_entry(xbuf + (i << 3), X);
  }
}

// Split-phase cooperative ROMix: the same per-wave pad layout as otd_scrypt_romix_coop, one phase per launch.
// Every wave of the chip is then in the same phase, so HBM sees pure sequential nt stores (launch 1) and then pure
// random full-line reads (launch 2) instead of the 1:1 mix that costs ~10% of bandwidth (tools/bench_hbm.hip:
// stores 5.8, reads 6.2, mixed 5.3-5.5 TB/s). Requires count <= grid * 256: each lane slot owns exactly one
// hash, whose pad must survive until the second launch.
template <int LCPOL, int PHASE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void otd_scrypt_romix_coop_phase(
    uint32_t count, uint4* __restrict__ xbuf, uint4* __restrict__ V) {
  __shared__ uint4 tiles[4 * 256];
  const uint64_t slot = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint32_t lane = uint32_t(slot & 63u);
  const uint64_t wave = (uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(slot >> 32))) << 26) |
                        uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(slot) >> 6));
  uint4* Vw = V + wave * (1024ull * 64u * 8u);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(Vw, (short)0, 1024 * 64 * 128, 0x00020000);
  uint4* tile = tiles + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * 256;
  if (slot < count) {  // count is a multiple of 64: whole waves take this branch together
    uint32_t X[32];
    load_entry(xbuf + (slot << 3), X);
    scrypt_romix_coop_phase<LCPOL, PHASE>(X, rs, tile, lane);
    store_entry(xbuf + (slot << 3), X);
  }
}

// Segmented cooperative ROMix: iterations [it0, it1) of the hash's 2048 (0..1023 write the pad, 1024..2047 look it
// up), X carried across launches in xbuf. The ROMix of one batch becomes `segments` launches of ~T/segments each
// (T ~ 32-64 ms with every wave slot of the chip held), so a kernel of another process -- the node's RCCL
// collective on its high-priority stream -- finds a free slot within one segment instead of one whole ROMix
// (parallel/comm_probe.py measures both the wait and the rate it costs: 2 x 128 B of X per lane per segment).
// Same residency rule as the split kernel: one hash per lane slot (count <= grid * 256).
template <int LCPOL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void otd_scrypt_romix_coop_seg(
    uint32_t count, uint4* __restrict__ xbuf, uint4* __restrict__ V, uint32_t it0, uint32_t it1,
    const otedama::HitSink sink) {
  __shared__ uint4 tiles[4 * 256];
  const uint64_t slot = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint32_t lane = uint32_t(slot & 63u);
  uint4* tile = tiles + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * 256;
  if (abort_newer(abort_peek(sink), sink.epoch)) return;  // stale work: pbkdf_out publishes nothing either
  // grid-stride over the batch's hashes (count is a multiple of 64: whole waves iterate together); a launch grid of
  // exactly the chip's resident blocks leaves no second round of blocks to straggle at each segment's end
  const uint64_t nslots = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t h = slot; h < count; h += nslots) {
    const uint64_t hw = (uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(h >> 32))) << 26) |
                        uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(h) >> 6));
    const __amdgpu_buffer_rsrc_t rh =
        __builtin_amdgcn_make_buffer_rsrc(V + hw * (1024ull * 64u * 8u), (short)0, 1024 * 64 * 128, 0x00020000);
    uint32_t X[32];
    load_entry(xbuf + (h << 3), X);
    const uint32_t w1 = it1 < 1024u ? it1 : 1024u;
    for (uint32_t i = it0; i < w1; ++i) {
      coop_store_entry(X, rh, tile, lane, i);
      blockmix(X);
    }
    for (uint32_t i = it0 > 1024u ? it0 : 1024u; i < it1; ++i) {
      coop_v4u R[4];
      coop_issue<LCPOL>(X, rh, tile, lane, R);
      coop_consume(X, tile, lane, R);
      blockmix(X);
    }
    store_entry(xbuf + (h << 3), X);
  }
}

// Two-stream cooperative ROMix: wave w owns hashes [128w, 128w+128) (lane l: 128w+l and 128w+64+l) and a
// 16 MiB pad region (8 MiB per stream). count is a multiple of 128 (launcher rounds up).
template <int LCPOL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void otd_scrypt_romix_coop2(
    uint32_t count, uint4* __restrict__ xbuf, uint4* __restrict__ V) {
  __shared__ uint4 tiles[4 * 256];
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave0 = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = (uint64_t(gridDim.x) * blockDim.x) >> 6;
  const uint64_t wslot = (uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(wave0 >> 32))) << 32) |
                         uint64_t(__builtin_amdgcn_readfirstlane(uint32_t(wave0)));
  uint4* VA = V + wslot * (2ull * 1024 * 64 * 8);
  uint4* VB = VA + 1024ull * 64 * 8;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(VA, (short)0, 1024 * 64 * 128, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(VB, (short)0, 1024 * 64 * 128, 0x00020000);
  uint4* tile = tiles + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * 256;
  for (uint64_t w = wslot; w * 128 < count; w += nwaves) {
    const uint64_t ia = w * 128 + lane, ib = ia + 64;
    uint32_t XA[32], XB[32];
    load_entry(xbuf + (ia << 3), XA);
    load_entry(xbuf + (ib << 3), XB);
    scrypt_romix_coop2<LCPOL>(XA, XB, rsA, rsB, tile, lane);
    store_entry(xbuf + (ia << 3), XA);
    store_entry(xbuf + (ib << 3), XB);
  }
}

// Same per-lane ROMix (gap 1) pinned to 8 waves/SIMD (64 VGPRs, no spill) for A/B against the
// compiler's default 67-VGPR / 7-wave allocation.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void otd_scrypt_romix_w8(
    uint32_t count, uint4* __restrict__ xbuf, uint4* __restrict__ V) {
  const uint64_t slot = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t nslots = uint64_t(gridDim.x) * blockDim.x;
  uint4* Vw = V + (slot >> 6) * (1024ull * 64u * 8u);
  const uint32_t lane = uint32_t(slot & 63u);
  for (uint64_t i = slot; i < count; i += nslots) {
    uint32_t X[32];
    load_entry(xbuf + (i << 3), X);
    scrypt_romix<1>(X, Vw, lane);
    store_entry(xbuf + (i << 3), X);
  }
}

// Hits (nonce) to `sink` (ops API: out[0] = candidate count, out[1..cap] = nonces). A batch whose abort word moved
// on publishes nothing: its ROMix stopped part way and xbuf holds unfinished states.
extern "C" __global__ __launch_bounds__(256) void otd_scrypt_pbkdf_out(const otedama::ScryptParams p, uint32_t base,
                                                                       uint32_t count, const uint4* __restrict__ xbuf,
                                                                       const otedama::HitSink sink) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  if (abort_newer(abort_peek(sink), sink.epoch)) return;
  uint32_t X[32];
  load_entry(xbuf + (uint64_t(i) << 3), X);
  const uint32_t h7 = scrypt_pbkdf_out(p, base + i, X);
  if (bswap(h7) <= p.target_hi) hit_publish(sink, base + i, 0u);
}

template __global__ void otd_scrypt_romix<1>(uint32_t, uint4*, uint4*);
template __global__ void otd_scrypt_romix<2>(uint32_t, uint4*, uint4*);
template __global__ void otd_scrypt_romix<4>(uint32_t, uint4*, uint4*);

namespace otedama {

// Scratchpad bytes for `grid` ROMix blocks of 256 lane slots at lookup gap `gap`.
uint64_t scrypt_scratch_bytes(int grid, int gap) {
  if (gap == kScryptCoop2) return uint64_t(grid) * 512ull * 1024ull * 128ull;  // 2 hashes per lane slot
  if (gap == kScryptCoop || gap == kScryptLaneW8 || gap == kScryptCoopSplit) gap = 1;
  return uint64_t(grid) * 256ull * (1024ull / uint64_t(gap)) * 128ull;
}

// OTEDAMA_SCRYPT_POLL=0: the ROMix write loop without its scalar abort polls (the A/B baseline; boundary polls only).
static bool scrypt_write_polls() {
  static const bool on = [] {
    const char* v = std::getenv("OTEDAMA_SCRYPT_POLL");
    return !(v && v[0] == '0');
  }();
  return on;
}

// OTEDAMA_SCRYPT_SEGMENTS=S (1..64): the cooperative ROMix of a batch as S launches (otd_scrypt_romix_coop_seg)
// when every lane slot holds one hash.
// Read at every launch (one environ scan per ~30 ms batch) so a test can switch it within one process.
// Unset = 0: the one-launch kernel. Set (1..64): the segmented kernel, S=1 included (its code alone, for the A/B).
static uint32_t scrypt_segments() {
  const char* v = std::getenv("OTEDAMA_SCRYPT_SEGMENTS");
  if (!v || !v[0]) return 0;
  const long x = std::strtol(v, nullptr, 10);
  return uint32_t(x < 1 ? 1 : (x > 64 ? 64 : x));
}

// OTEDAMA_SCRYPT_SEG_GRID caps the segmented kernel's launch grid: "resident" = the chip's resident blocks (8 per CU
// at 8 waves/SIMD), N = N blocks; each lane slot then walks several hashes per segment. Unset: the allocation grid
// (one hash per lane slot).
static int scrypt_seg_grid(int grid) {
  const char* v = std::getenv("OTEDAMA_SCRYPT_SEG_GRID");
  if (!v || !v[0]) return grid;
  int cap = 0;
  if (std::strcmp(v, "resident") == 0) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      return grid;
    cap = cus * 8;
  } else {
    cap = int(std::strtol(v, nullptr, 10));
  }
  return cap > 0 && cap < grid ? cap : grid;
}

// xbuf: count * 128 bytes. scratch: scrypt_scratch_bytes(grid, gap).
// gap: 1/2/4 = per-lane ROMix with that lookup gap; kScryptCoop = lane-cooperative ROMix (gap 1).
hipError_t launch_scrypt_search(const ScryptParams& p, uint32_t base, uint32_t count, void* xbuf, void* scratch,
                                int gap, const HitSink& sink, int grid, hipStream_t stream) {
  uint4* X = static_cast<uint4*>(xbuf);
  uint4* V = static_cast<uint4*>(scratch);
  const int eg = int((count + 255) / 256);
  // The cooperative kernel runs whole waves (shfl + octet loads): round its count up to 64 lanes. xbuf is
  // allocated in multiples of 256 lanes, and lanes past `count` are ignored by pbkdf_out.
  const uint32_t count64 = (count + 63u) & ~63u;
  // Refuse before anything is enqueued: the split ROMix holds one hash per lane slot across its two launches.
  if (gap == kScryptCoopSplit && uint64_t(count64) > uint64_t(grid) * 256u) return hipErrorInvalidValue;
  hipLaunchKernelGGL(otd_scrypt_pbkdf_in, dim3(eg), dim3(256), 0, stream, p, base, count, X);
  switch (gap) {
    case kScryptCoop:  // nt lookups: +0.5-1% over default-policy loads (profiles/r1/scrypt_romix_ab.md)
      if (scrypt_segments() > 0 && uint64_t(count64) <= uint64_t(grid) * 256u) {
        const uint32_t S = scrypt_segments();
        const int sg = scrypt_seg_grid(grid);
        for (uint32_t k = 0; k < S; ++k)
          hipLaunchKernelGGL(otd_scrypt_romix_coop_seg<2>, dim3(sg), dim3(256), 0, stream, count64, X, V,
                             2048u * k / S, 2048u * (k + 1) / S, sink);
      } else if (scrypt_write_polls())
        hipLaunchKernelGGL((otd_scrypt_romix_coop<2, 64>), dim3(grid), dim3(256), 0, stream, count64, X, V, sink);
      else
        hipLaunchKernelGGL((otd_scrypt_romix_coop<2, 1024>), dim3(grid), dim3(256), 0, stream, count64, X, V, sink);
      break;
    case kScryptLaneW8:
      hipLaunchKernelGGL(otd_scrypt_romix_w8, dim3(grid), dim3(256), 0, stream, count, X, V);
      break;
    case kScryptCoopSplit:
      hipLaunchKernelGGL((otd_scrypt_romix_coop_phase<2, 1>), dim3(grid), dim3(256), 0, stream, count64, X, V);
      hipLaunchKernelGGL((otd_scrypt_romix_coop_phase<2, 2>), dim3(grid), dim3(256), 0, stream, count64, X, V);
      break;
    case kScryptCoop2:
      hipLaunchKernelGGL(otd_scrypt_romix_coop2<2>, dim3(grid), dim3(256), 0, stream, (count + 127u) & ~127u, X, V);
      break;
    case 1: hipLaunchKernelGGL(otd_scrypt_romix<1>, dim3(grid), dim3(256), 0, stream, count, X, V); break;
    case 2: hipLaunchKernelGGL(otd_scrypt_romix<2>, dim3(grid), dim3(256), 0, stream, count, X, V); break;
    case 4: hipLaunchKernelGGL(otd_scrypt_romix<4>, dim3(grid), dim3(256), 0, stream, count, X, V); break;
    default: return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(otd_scrypt_pbkdf_out, dim3(eg), dim3(256), 0, stream, p, base, count, X, sink);
  return hipGetLastError();
}

}  // namespace otedama
