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

// out[0]: candidate count (may exceed cap); out[1..cap]: nonces (header byte order).
// Nonces are header-order values (bytes 76..79 little-endian); the kernel feeds
// W3 = bswap(nonce) (one v_perm per nonce) so base/count index the nonce itself.
extern "C" __global__ __launch_bounds__(256) void otd_sha256d_search(
    const otedama::Sha256dParams p, uint32_t base, uint64_t count, uint32_t* __restrict__ out,
    uint32_t cap) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint64_t off = tid; off < count; off += stride) {
    const uint32_t nonce = base + static_cast<uint32_t>(off);
    const uint32_t w3 = __builtin_bswap32(nonce);
    const uint32_t h7 = sha256d_h7(p, w3);
    if (__builtin_bswap32(h7) <= p.target_hi) {
      const uint32_t slot = atomicAdd(out, 1u);
      if (slot < cap) out[1 + slot] = nonce;
    }
  }
}

// ---------------------------------------------------------------- K-variant search
// K header variants that differ only in block 1 (BIP320 version rolling; SV2 standard channels) share
// block 2 of the first hash — merkle tail, ntime, nbits, nonce — so they share its message schedule
// W16..W63 (~460 VALU per nonce): each lane computes W once and advances K states in lockstep
// (the overt-AsicBoost observation, applied per lane). Hash 2 depends on each variant's digest and
// runs per variant. Every variant still scans the full nonce range with its own fixed midstate.
namespace {

template <int K>
__device__ __forceinline__ void sha256d_h7_k(const otedama::Sha256dParamsK& p, uint32_t w3, uint32_t h7[K]) {
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
    const otedama::Sha256dVariant& q = p.var[v];
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
#pragma unroll
  for (int v = 0; v < K; ++v) {
    const otedama::Sha256dVariant& q = p.var[v];
    uint32_t X[61];
    X[0] = q.mid[0] + A[v]; X[1] = q.mid[1] + B[v]; X[2] = q.mid[2] + C[v]; X[3] = q.mid[3] + D[v];
    X[4] = q.mid[4] + E[v]; X[5] = q.mid[5] + F[v]; X[6] = q.mid[6] + G[v]; X[7] = q.mid[7] + H[v];
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
    h7[v] = e + kIV[7];
  }
}

}  // namespace

// out[0]: count; out[1 + 2*i] = nonce, out[2 + 2*i] = variant index (0..K-1).
template <int K>
__global__ __launch_bounds__(256) void otd_sha256d_search_k(const otedama::Sha256dParamsK p, uint32_t base,
                                                            uint64_t count, uint32_t* __restrict__ out, uint32_t cap) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint64_t off = tid; off < count; off += stride) {
    const uint32_t nonce = base + static_cast<uint32_t>(off);
    uint32_t h7[K];
    sha256d_h7_k<K>(p, __builtin_bswap32(nonce), h7);
#pragma unroll
    for (int v = 0; v < K; ++v) {
      if (__builtin_bswap32(h7[v]) <= p.target_hi) {
        const uint32_t slot = atomicAdd(out, 1u);
        if (slot < cap) {
          out[1 + 2 * slot] = nonce;
          out[2 + 2 * slot] = (uint32_t)v;
        }
      }
    }
  }
}
template __global__ void otd_sha256d_search_k<2>(const otedama::Sha256dParamsK, uint32_t, uint64_t, uint32_t*, uint32_t);
template __global__ void otd_sha256d_search_k<3>(const otedama::Sha256dParamsK, uint32_t, uint64_t, uint32_t*, uint32_t);
template __global__ void otd_sha256d_search_k<4>(const otedama::Sha256dParamsK, uint32_t, uint64_t, uint32_t*, uint32_t);

namespace otedama {

hipError_t launch_sha256d_search(const Sha256dParams& p, uint32_t base, uint64_t count, uint32_t* out,
                                 uint32_t cap, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(otd_sha256d_search, dim3(grid), dim3(256), 0, stream, p, base, count, out, cap);
  return hipGetLastError();
}

hipError_t launch_sha256d_search_k(const Sha256dParamsK& p, uint32_t base, uint64_t count, uint32_t* out, uint32_t cap,
                                   int grid, hipStream_t stream) {
  switch (p.k) {
    case 2: hipLaunchKernelGGL(otd_sha256d_search_k<2>, dim3(grid), dim3(256), 0, stream, p, base, count, out, cap); break;
    case 3: hipLaunchKernelGGL(otd_sha256d_search_k<3>, dim3(grid), dim3(256), 0, stream, p, base, count, out, cap); break;
    case 4: hipLaunchKernelGGL(otd_sha256d_search_k<4>, dim3(grid), dim3(256), 0, stream, p, base, count, out, cap); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace otedama
