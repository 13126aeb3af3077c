// sha256d_search — per-lane SHA-256d nonce search for gfx950 (CDNA4).
//
// Replaces the reference's CPU grind loop (internal/miner/worker.go:216-282 and
// internal/miner/sha256d.go:107-117: 3 compressions per nonce, per-hash atomic)
// with a VALU-bound kernel:
//   * block 1 (header bytes 0..63) is folded into a midstate on the host, as are
//     rounds 0..2 of block 2 and W16/W17 (job.h);
//   * round 3 is two adds (the nonce is W3); W4..W15 are literal padding so the
//     schedule constant-folds;
//   * the second SHA-256 runs only to round 60 and only computes `e` in rounds
//     57..60, because H7 = IV7 + e60 is all the early-reject needs;
//   * rotations are v_alignbit_b32, Ch/Maj/xor3 are single v_bitop3_b32 ops
//     (CDNA4), sums fold to v_add3_u32; every nonce-invariant value is
//     wave-uniform and stays in SGPRs, so VGPR use stays low (>= 6 waves/SIMD);
//   * no memory traffic except an atomic append per candidate: hashes are
//     counted per launch on the host, not per nonce.
// Candidates (bswap(H7) <= target_hi) are re-verified on the host with the
// full 256-bit compare, so a target_hi tie can never produce a false share.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cdna_bitops.h"
#include "hitsink_dev.h"
#include "otedama/job.h"

namespace {

using namespace otedama_dev;
constexpr const uint32_t* kIV = kSha256IVd;
__device__ __forceinline__ constexpr uint32_t Kf(int i) { return sha256_k(i); }

// SHA-256d of one nonce; returns H7 (last state word of the second hash).
__device__ __forceinline__ uint32_t sha256d_h7(const otedama::Sha256dParams& p, uint32_t w3) {
  // ---- hash 1, block 2: rounds 3..63 ----
  uint32_t W[64];
  W[0] = p.w0; W[1] = p.w1; W[2] = p.w2; W[3] = w3;
  W[4] = 0x80000000u;
#pragma unroll
  for (int i = 5; i < 15; ++i) W[i] = 0u;
  W[15] = 640u;
  W[16] = p.w16;
  W[17] = p.w17;

  uint32_t a = p.st3[0], b = p.st3[1], c = p.st3[2], d = p.st3[3];
  uint32_t e = p.st3[4], f = p.st3[5], g = p.st3[6], h = p.st3[7];
  {  // round 3: T1 = pre3 + nonce
    const uint32_t t1 = p.pre3 + w3;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + p.t2_3;
  }
#pragma unroll
  for (int t = 4; t < 64; ++t) {
    // W[i] is lane-varying iff i == 3 (nonce) or i >= 18.
    if (t >= 18) W[t] = ss1(W[t - 2], t >= 20) + W[t - 7] + ss0(W[t - 15], t == 18 || t >= 33) + W[t - 16];
    const uint32_t t1 = h + bS1(e) + ch(e, f, g) + (Kf(t) + W[t]);
    const uint32_t t2 = bS0(a) + maj(a, b, c);
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  // ---- hash 2: one block, W0..7 = digest, constant padding ----
  uint32_t X[61];
  X[0] = p.mid[0] + a; X[1] = p.mid[1] + b; X[2] = p.mid[2] + c; X[3] = p.mid[3] + d;
  X[4] = p.mid[4] + e; X[5] = p.mid[5] + f; X[6] = p.mid[6] + g; X[7] = p.mid[7] + h;
  X[8] = 0x80000000u;
#pragma unroll
  for (int i = 9; i < 15; ++i) X[i] = 0u;
  X[15] = 256u;
  a = kIV[0]; b = kIV[1]; c = kIV[2]; d = kIV[3];
  e = kIV[4]; f = kIV[5]; g = kIV[6]; h = kIV[7];
#pragma unroll
  for (int t = 0; t < 61; ++t) {
    // X[i] is lane-varying iff i <= 7 or i >= 16 (X8..X15 are padding constants).
    if (t >= 16) X[t] = ss1(X[t - 2], t >= 18) + X[t - 7] + ss0(X[t - 15], t <= 22 || t >= 31) + X[t - 16];
    const uint32_t t1 = h + bS1(e) + ch(e, f, g) + (Kf(t) + X[t]);
    const uint32_t ne = d + t1;
    // a is dead after round 56 (only d of round 60 = a56 reaches e60); DCE drops it.
    const uint32_t na = t1 + bS0(a) + maj(a, b, c);
    h = g; g = f; f = e; e = ne; d = c; c = b; b = a; a = na;
  }
  return e + kIV[7];
}

}  // namespace

// Hits go to `sink` (otedama/hitsink.h; ops API: out[0] = count, out[1..cap] = nonces in header byte order).
// Nonces are header-order values (bytes 76..79 little-endian); the kernel feeds
// W3 = bswap(nonce) (one v_perm per nonce) so base/count index the nonce itself.
// A trip here is one hash per lane (~1 us per wave), so the abort word is polled every kAbortTrips trips.
// This kernel polls with abort_peek (wave-uniform right after the load), not the split issue/seen form of the
// multi-variant kernels: in one process on the MI355X the split form ran 1.8-2.2% slower here at every grid
// (and peek matched no poll at all), at the same 51/50 VGPRs and 7 waves/SIMD (profiles/r3/ad_single).
constexpr uint32_t kAbortTrips = 32;
extern "C" __global__ __launch_bounds__(256) void otd_sha256d_search(
    const otedama::Sha256dParams p, uint32_t base, uint64_t count, const otedama::HitSink sink) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t stride = gridDim.x * blockDim.x;
  uint32_t ab = abort_peek(sink), trip = 0;
  for (uint64_t off = tid; off < count; off += stride) {
    if (++trip == kAbortTrips) {
      if (abort_newer(ab, sink.epoch)) break;
      ab = abort_peek(sink);
      trip = 0;
    }
    const uint32_t nonce = base + static_cast<uint32_t>(off);
    const uint32_t w3 = __builtin_bswap32(nonce);
    const uint32_t h7 = sha256d_h7(p, w3);
    if (__builtin_bswap32(h7) <= p.target_hi) hit_publish(sink, nonce, 0u);
  }
}

// ---------------------------------------------------------------- K-variant search
// K header variants that differ only in block 1 (BIP320 version rolling; SV2 standard channels) share
// block 2 of the first hash — merkle tail, ntime, nbits, nonce — so they share its message schedule
// W16..W63 (~460 VALU per nonce): each lane computes W once and advances K states in lockstep
// (the overt-AsicBoost observation, applied per lane). Hash 2 depends on each variant's digest and
// runs per variant. Every variant still scans the full nonce range with its own fixed midstate.
//
// Register budget (hipcc -Rpass-analysis=kernel-resource-usage, gfx950): the per-variant constants
// (18 words each) are re-read from the kernarg segment with s_load on every nonce instead of being
// hoisted out of the nonce loop. Hoisted, they overflow the 102 SGPRs and spill into VGPR lanes
// (133 v_readlane/v_writelane per loop trip at K=4, 700 at K=8). Re-read, K=4 needs 79 VGPRs and no
// lane spills, and K=8 fits 121 VGPRs (4 waves/SIMD). Static VALU per variant-hash: K=4 2202, K=8 2146,
// K=16 2115. The file is built with a raised -pragma-unroll-threshold (otedama_amd/_build.py): at
// K >= 6 the round loop is otherwise left rolled and W[]/state arrays go to scratch.
namespace {

using KParamsK = const __attribute__((address_space(4))) otedama::Sha256dParamsK;

// Hash 2 of one variant from its first-hash state: returns H7.
template <class M>
__device__ __forceinline__ uint32_t sha256_h7_of_state(const M& mid, uint32_t a0, uint32_t b0, uint32_t c0,
                                                       uint32_t d0, uint32_t e0, uint32_t f0, uint32_t g0, uint32_t h0) {
  uint32_t X[61];
  X[0] = mid[0] + a0; X[1] = mid[1] + b0; X[2] = mid[2] + c0; X[3] = mid[3] + d0;
  X[4] = mid[4] + e0; X[5] = mid[5] + f0; X[6] = mid[6] + g0; X[7] = mid[7] + h0;
  X[8] = 0x80000000u;
#pragma unroll
  for (int i = 9; i < 15; ++i) X[i] = 0u;
  X[15] = 256u;
  uint32_t a = kIV[0], b = kIV[1], c = kIV[2], d = kIV[3], e = kIV[4], f = kIV[5], g = kIV[6], h = kIV[7];
#pragma unroll
  for (int t = 0; t < 61; ++t) {
    if (t >= 16) X[t] = ss1(X[t - 2], t >= 18) + X[t - 7] + ss0(X[t - 15], t <= 22 || t >= 31) + X[t - 16];
    const uint32_t t1 = h + bS1(e) + ch(e, f, g) + (Kf(t) + X[t]);
    const uint32_t ne = d + t1;
    const uint32_t na = t1 + bS0(a) + maj(a, b, c);
    h = g; g = f; f = e; e = ne; d = c; c = b; b = a; a = na;
  }
  return e + kIV[7];
}

// Hash 2 of variants V..K-1 by compile-time recursion: a runtime loop over the variants is not
// unrolled for large K, and its A[v]..H[v] indexing would then live in scratch.
template <int V, int K>
__device__ __forceinline__ void hash2_all(KParamsK& p, const uint32_t* A, const uint32_t* B, const uint32_t* C,
                                          const uint32_t* D, const uint32_t* E, const uint32_t* F, const uint32_t* G,
                                          const uint32_t* H, uint32_t* h7) {
  if constexpr (V < K) {
    h7[V] = sha256_h7_of_state(p.var[V].mid, A[V], B[V], C[V], D[V], E[V], F[V], G[V], H[V]);
    hash2_all<V + 1, K>(p, A, B, C, D, E, F, G, H, h7);
  }
}

template <int K>
__device__ __forceinline__ void sha256d_h7_k(KParamsK& p, uint32_t w3, uint32_t h7[K]) {
  uint32_t W[64];
  W[0] = p.w0; W[1] = p.w1; W[2] = p.w2; W[3] = w3;
  W[4] = 0x80000000u;
#pragma unroll
  for (int i = 5; i < 15; ++i) W[i] = 0u;
  W[15] = 640u;
  W[16] = p.w16;
  W[17] = p.w17;
  uint32_t A[K], B[K], C[K], D[K], E[K], F[K], G[K], H[K];
#pragma unroll
  for (int v = 0; v < K; ++v) {  // round 3: T1 = pre3 + nonce
    const auto& q = p.var[v];
    const uint32_t t1 = q.pre3 + w3;
    H[v] = q.st3[6]; G[v] = q.st3[5]; F[v] = q.st3[4]; E[v] = q.st3[3] + t1;
    D[v] = q.st3[2]; C[v] = q.st3[1]; B[v] = q.st3[0]; A[v] = t1 + q.t2_3;
  }
#pragma unroll
  for (int t = 4; t < 64; ++t) {
    if (t >= 18) W[t] = ss1(W[t - 2], t >= 20) + W[t - 7] + ss0(W[t - 15], t == 18 || t >= 33) + W[t - 16];
    const uint32_t kw = Kf(t) + W[t];
#pragma unroll
    for (int v = 0; v < K; ++v) {
      const uint32_t t1 = H[v] + bS1(E[v]) + ch(E[v], F[v], G[v]) + kw;
      const uint32_t t2 = bS0(A[v]) + maj(A[v], B[v], C[v]);
      H[v] = G[v]; G[v] = F[v]; F[v] = E[v]; E[v] = D[v] + t1; D[v] = C[v]; C[v] = B[v]; B[v] = A[v]; A[v] = t1 + t2;
    }
  }
  hash2_all<0, K>(p, A, B, C, D, E, F, G, H, h7);
}

}  // namespace

// Hits: (nonce, variant index 0..K-1) to `sink` (ops API: out[0] = count, out[1 + 2*i] = nonce, out[2 + 2*i] =
// variant). One trip is K hashes per lane: the abort word is polled every kAbortTrips / K trips.
template <int K>
__global__ __launch_bounds__(256) void otd_sha256d_search_k(const otedama::Sha256dParamsK p, uint32_t base,
                                                            uint64_t count, const otedama::HitSink sink) {
  (void)p;  // read through the kernarg segment pointer below (p is the first kernel argument, offset 0)
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t stride = gridDim.x * blockDim.x;
  constexpr uint32_t kTrips = kAbortTrips / K > 0 ? kAbortTrips / K : 1;
  uint32_t ab = abort_issue(sink), trip = 0;
  for (uint64_t off = tid; off < count; off += stride) {
    if (++trip == kTrips) {
      if (abort_seen(ab, sink.epoch)) break;
      ab = abort_issue(sink);
      trip = 0;
    }
    const uint32_t nonce = base + static_cast<uint32_t>(off);
    // Opaque per trip: the compiler cannot hoist the (scalar) parameter loads out of the loop.
    KParamsK* pp = (KParamsK*)(__builtin_amdgcn_kernarg_segment_ptr());
    asm volatile("" : "+s"(pp));
    uint32_t h7[K];
    sha256d_h7_k<K>(*pp, __builtin_bswap32(nonce), h7);
#pragma unroll
    for (int v = 0; v < K; ++v) {
      if (__builtin_bswap32(h7[v]) <= p.target_hi) hit_publish(sink, nonce, uint32_t(v));
    }
  }
}
#define OTD_SHA_K_INSTANCE(K) \
  template __global__ void otd_sha256d_search_k<K>(const otedama::Sha256dParamsK, uint32_t, uint64_t, const otedama::HitSink);
OTD_SHA_K_INSTANCE(2)
OTD_SHA_K_INSTANCE(3)
OTD_SHA_K_INSTANCE(4)
OTD_SHA_K_INSTANCE(6)
OTD_SHA_K_INSTANCE(8)
OTD_SHA_K_INSTANCE(12)
OTD_SHA_K_INSTANCE(16)
#undef OTD_SHA_K_INSTANCE

namespace otedama {

hipError_t launch_sha256d_search(const Sha256dParams& p, uint32_t base, uint64_t count, const HitSink& sink, int grid,
                                 hipStream_t stream) {
  hipLaunchKernelGGL(otd_sha256d_search, dim3(grid), dim3(256), 0, stream, p, base, count, sink);
  return hipGetLastError();
}

hipError_t launch_sha256d_search_k(const Sha256dParamsK& p, uint32_t base, uint64_t count, const HitSink& sink, int grid,
                                   hipStream_t stream) {
  switch (p.k) {
#define OTD_SHA_K_CASE(K) \
  case K: hipLaunchKernelGGL(otd_sha256d_search_k<K>, dim3(grid), dim3(256), 0, stream, p, base, count, sink); break;
    OTD_SHA_K_CASE(2) OTD_SHA_K_CASE(3) OTD_SHA_K_CASE(4) OTD_SHA_K_CASE(6) OTD_SHA_K_CASE(8) OTD_SHA_K_CASE(12)
    OTD_SHA_K_CASE(16)
#undef OTD_SHA_K_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace otedama
