// sha256d_search_v — version-parallel SHA-256d search: the 64 lanes of a wave are 64 BIP320 version variants of
// one header, and the wave walks the nonce space together.
//
// Why: the K-variant kernel (sha256d_search.hip) shares the first hash's block-2 message schedule among K
// variants inside a lane, but still computes that schedule on the VALU once per lane-nonce (~58 VALU per
// variant-hash at K=8). Here the nonce is wave-uniform, so the whole schedule W18..W63 and every K[t]+W[t]
// are wave-uniform too: the compiler keeps them in SGPRs and computes them on the scalar ALU, which issues
// in parallel with other waves' VALU work (one SALU and one VALU per SIMD issue slot). What is left on the
// VALU per variant-hash is the 61 rounds of hash 1, the digest add and hash 2 — no schedule, no K-fold state
// arrays (one state per lane, ~60 VGPRs, 8 waves/SIMD instead of 4).
//
// Variants: lane l of variant group g hashes the header whose block 1 (version, prev-hash, merkle head)
// gives vars[64*g + l] (midstate, state after rounds 0..2 of block 2, round-3 constants; job.h). All
// variants of one launch share block 2 (merkle tail, ntime, nbits), i.e. they differ only in the version.
// Nonce walk: W3 (the big-endian nonce word) runs over [base, base + count); the nonce written to a header
// is bswap(W3), reported as such. Launches that tile W3 tile the nonce space.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cdna_bitops.h"
#include "hitsink_dev.h"
#include "otedama/job.h"

namespace {

using namespace otedama_dev;
constexpr const uint32_t* kIVv = kSha256IVd;

// Scalar (wave-uniform) schedule helpers. The scalar ALU has no rotate and LLVM turns a C rotate into a funnel
// shift that only selects to v_alignbit, which would drag the whole schedule onto the VALU. So the rotates are
// spelled as s_lshr_b64 of the pair (x:x) (the low half is rotr(x, n)); xors and adds of the SGPR results stay
// scalar on their own.
template <int N>
__device__ __forceinline__ uint32_t srotr(uint64_t xx) {
  uint64_t r;
  asm("s_lshr_b64 %0, %1, %2" : "=s"(r) : "s"(xx), "n"(N));
  return static_cast<uint32_t>(r);
}
__device__ __forceinline__ uint64_t spair(uint32_t x) { return (static_cast<uint64_t>(x) << 32) | x; }
__device__ __forceinline__ uint32_t sss0(uint32_t x) {
  const uint64_t xx = spair(x);
  return srotr<7>(xx) ^ srotr<18>(xx) ^ (x >> 3);
}
__device__ __forceinline__ uint32_t sss1(uint32_t x) {
  const uint64_t xx = spair(x);
  return srotr<17>(xx) ^ srotr<19>(xx) ^ (x >> 10);
}

using VarPtr = const otedama::Sha256dVariant* __restrict__;

}  // namespace

// Hits (nonce in header byte order, variant index) go to `sink` (otedama/hitsink.h): the host-coherent ring of the
// native miner, or out[0] = count, out[1 + 2i] = nonce, out[2 + 2i] = variant for the ops API.
// Grid contract (checked on the host): the wave count gridDim.x * blockDim.x / 64 is a multiple of p.groups, so every
// variant group gets the same number of waves and each wave's nonce stride is uniform.
// MINW = 0: default build, 63 VGPRs / 106 SGPRs -> 7 waves/SIMD (SGPR-limited);
// MINW = 8: 8 waves/SIMD, the SGPR budget drops and more schedule words live in VGPR lanes (v_readlane).
// The body sits in the kernel itself: routed through a device function taking the params by reference, the
// compiler forms fewer v_add3 with the SGPR K+W word (2117 instead of 2084 VALU per hash).
template <int MINW>
__global__ __launch_bounds__(256, MINW > 0 ? MINW : 1) void otd_sha256d_search_v(
    const otedama::Sha256dParamsV p, VarPtr vars, uint32_t base, uint64_t count, const otedama::HitSink sink) {
  const uint32_t wpb = blockDim.x >> 6;  // waves per block (256 or 64 threads)
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * wpb + (threadIdx.x >> 6));
  const uint32_t waves = gridDim.x * wpb;
  const uint32_t groups = p.groups;
  const uint32_t g = wave % groups;
  const uint32_t first = wave / groups;
  const uint32_t stride = waves / groups;
  const uint32_t vi = g * 64u + (threadIdx.x & 63u);
  const otedama::Sha256dVariant& v = vars[vi];
  uint32_t mid[8], st3[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mid[i] = v.mid[i];
    st3[i] = v.st3[i];
  }
  const uint32_t pre3 = v.pre3, t2_3 = v.t2_3;

  // Abort poll, one per grid-stride iteration: the load for the next check is issued at the top of each trip and
  // only waited on at the next trip's top, so its latency hides under a whole iteration of hashing.
  uint32_t ab = abort_issue(sink);
  for (uint64_t off = first; off < count; off += stride) {
    if (abort_seen(ab, sink.epoch)) break;
    ab = abort_issue(sink);
    const uint32_t w3 = base + static_cast<uint32_t>(off);  // wave-uniform
    // ---- hash 1, block 2: rounds 3..63 (schedule on the scalar unit) ----
    uint32_t W[64];
    W[0] = p.w0; W[1] = p.w1; W[2] = p.w2; W[3] = w3;
    W[4] = 0x80000000u;
#pragma unroll
    for (int i = 5; i < 15; ++i) W[i] = 0u;
    W[15] = 640u;
    W[16] = p.w16;
    W[17] = p.w17;
    const uint32_t t1_3 = pre3 + w3;
    uint32_t h = st3[6], gg = st3[5], f = st3[4], e = st3[3] + t1_3;
    uint32_t d = st3[2], c = st3[1], b = st3[0], a = t1_3 + t2_3;
#pragma unroll
    for (int t = 4; t < 64; ++t) {
      if (t >= 18) W[t] = sss1(W[t - 2]) + W[t - 7] + sss0(W[t - 15]) + W[t - 16];
      const uint32_t kw = sha256_k(t) + W[t];  // SGPR
      const uint32_t t1 = h + bS1(e) + ch(e, f, gg) + kw;
      const uint32_t t2 = bS0(a) + maj(a, b, c);
      h = gg; gg = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
      __builtin_amdgcn_sched_barrier(0);  // keep the scalar schedule one round ahead at most (SGPR budget)
    }
    // ---- hash 2: one block, X0..7 = digest, constant padding; only e of rounds 57..60 is live ----
    uint32_t X[61];
    X[0] = mid[0] + a; X[1] = mid[1] + b; X[2] = mid[2] + c; X[3] = mid[3] + d;
    X[4] = mid[4] + e; X[5] = mid[5] + f; X[6] = mid[6] + gg; X[7] = mid[7] + h;
    X[8] = 0x80000000u;
#pragma unroll
    for (int i = 9; i < 15; ++i) X[i] = 0u;
    X[15] = 256u;
    a = kIVv[0]; b = kIVv[1]; c = kIVv[2]; d = kIVv[3];
    e = kIVv[4]; f = kIVv[5]; gg = kIVv[6]; h = kIVv[7];
#pragma unroll
    for (int t = 0; t < 61; ++t) {
      if (t >= 16) X[t] = ss1(X[t - 2], t >= 18) + X[t - 7] + ss0(X[t - 15], t <= 22 || t >= 31) + X[t - 16];
      const uint32_t t1 = h + bS1(e) + ch(e, f, gg) + (sha256_k(t) + X[t]);
      const uint32_t ne = d + t1;
      const uint32_t na = t1 + bS0(a) + maj(a, b, c);
      h = gg; gg = f; f = e; e = ne; d = c; c = b; b = a; a = na;
    }
    const uint32_t h7 = e + kIVv[7];
    if (__builtin_bswap32(h7) <= p.target_hi) hit_publish(sink, __builtin_bswap32(w3), vi);
  }
}

template __global__ void otd_sha256d_search_v<0>(const otedama::Sha256dParamsV, VarPtr, uint32_t, uint64_t,
                                                   const otedama::HitSink);
template __global__ void otd_sha256d_search_v<8>(const otedama::Sha256dParamsV, VarPtr, uint32_t, uint64_t,
                                                   const otedama::HitSink);


// NC variants per lane (lane l of group g: variants 64*NC*g + 64c + l, c < NC), same nonce: all chains use the one
// scalar schedule, so the SALU work per hash drops NC-fold, and the independent round chains give each wave ILP at
// lower occupancy. NC = 2: 111 VGPRs, 4 waves/SIMD (MINW = 5: 96 VGPRs, 5 waves); NC = 3: 157 VGPRs, 3 waves;
// NC = 4: 203 VGPRs, 2 waves. p.groups counts groups of 64*NC variants.
// POLL picks the abort-poll form: 0 split issue/seen every trip (production), 1 abort_peek every trip, 2 none.
// Only 0 is instantiated here; tools/sha_v_ab.hip instantiates the others for same-process A/B runs.
template <int NC, int MINW, int POLL = 0>
__global__ __launch_bounds__(256, MINW > 0 ? MINW : 1) void otd_sha256d_search_vn(
    const otedama::Sha256dParamsV p, VarPtr vars, uint32_t base, uint64_t count, const otedama::HitSink sink) {
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * wpb + (threadIdx.x >> 6));
  const uint32_t waves = gridDim.x * wpb;
  const uint32_t groups = p.groups;
  const uint32_t g = wave % groups;
  const uint32_t first = wave / groups;
  const uint32_t stride = waves / groups;
  uint32_t vi[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) vi[c] = g * (64u * NC) + 64u * c + (threadIdx.x & 63u);
  uint32_t mid[NC][8], st3[NC][8], pre3[NC], t2_3[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const otedama::Sha256dVariant& v = vars[vi[c]];
#pragma unroll
    for (int i = 0; i < 8; ++i) { mid[c][i] = v.mid[i]; st3[c][i] = v.st3[i]; }
    pre3[c] = v.pre3; t2_3[c] = v.t2_3;
  }
  // as in otd_sha256d_search_v: one poll per trip, latency hidden by the trip
  uint32_t ab = POLL == 1 ? abort_peek(sink) : abort_issue(sink);
  for (uint64_t off = first; off < count; off += stride) {
    if constexpr (POLL == 0) {
      if (abort_seen(ab, sink.epoch)) break;
      ab = abort_issue(sink);
    } else if constexpr (POLL == 1) {
      if (abort_newer(ab, sink.epoch)) break;
      ab = abort_peek(sink);
    }
    const uint32_t w3 = base + static_cast<uint32_t>(off);
    uint32_t W[64];
    W[0] = p.w0; W[1] = p.w1; W[2] = p.w2; W[3] = w3;
    W[4] = 0x80000000u;
#pragma unroll
    for (int i = 5; i < 15; ++i) W[i] = 0u;
    W[15] = 640u;
    W[16] = p.w16;
    W[17] = p.w17;
    uint32_t a[NC], b[NC], c_[NC], d[NC], e[NC], f[NC], gg[NC], h[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const uint32_t t1_3 = pre3[c] + w3;
      h[c] = st3[c][6]; gg[c] = st3[c][5]; f[c] = st3[c][4]; e[c] = st3[c][3] + t1_3;
      d[c] = st3[c][2]; c_[c] = st3[c][1]; b[c] = st3[c][0]; a[c] = t1_3 + t2_3[c];
    }
#pragma unroll
    for (int t = 4; t < 64; ++t) {
      if (t >= 18) W[t] = sss1(W[t - 2]) + W[t - 7] + sss0(W[t - 15]) + W[t - 16];
      const uint32_t kw = sha256_k(t) + W[t];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const uint32_t t1 = h[c] + bS1(e[c]) + ch(e[c], f[c], gg[c]) + kw;
        const uint32_t t2 = bS0(a[c]) + maj(a[c], b[c], c_[c]);
        h[c] = gg[c]; gg[c] = f[c]; f[c] = e[c]; e[c] = d[c] + t1; d[c] = c_[c]; c_[c] = b[c]; b[c] = a[c]; a[c] = t1 + t2;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    uint32_t X[NC][61];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      X[c][0] = mid[c][0] + a[c]; X[c][1] = mid[c][1] + b[c]; X[c][2] = mid[c][2] + c_[c]; X[c][3] = mid[c][3] + d[c];
      X[c][4] = mid[c][4] + e[c]; X[c][5] = mid[c][5] + f[c]; X[c][6] = mid[c][6] + gg[c]; X[c][7] = mid[c][7] + h[c];
      X[c][8] = 0x80000000u;
#pragma unroll
      for (int i = 9; i < 15; ++i) X[c][i] = 0u;
      X[c][15] = 256u;
      a[c] = kIVv[0]; b[c] = kIVv[1]; c_[c] = kIVv[2]; d[c] = kIVv[3];
      e[c] = kIVv[4]; f[c] = kIVv[5]; gg[c] = kIVv[6]; h[c] = kIVv[7];
    }
#pragma unroll
    for (int t = 0; t < 61; ++t) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if (t >= 16) X[c][t] = ss1(X[c][t - 2], t >= 18) + X[c][t - 7] + ss0(X[c][t - 15], t <= 22 || t >= 31) + X[c][t - 16];
        const uint32_t t1 = h[c] + bS1(e[c]) + ch(e[c], f[c], gg[c]) + (sha256_k(t) + X[c][t]);
        const uint32_t ne = d[c] + t1;
        const uint32_t na = t1 + bS0(a[c]) + maj(a[c], b[c], c_[c]);
        h[c] = gg[c]; gg[c] = f[c]; f[c] = e[c]; e[c] = ne; d[c] = c_[c]; c_[c] = b[c]; b[c] = a[c]; a[c] = na;
      }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const uint32_t h7 = e[c] + kIVv[7];
      if (__builtin_bswap32(h7) <= p.target_hi) hit_publish(sink, __builtin_bswap32(w3), vi[c]);
    }
  }
}

template __global__ void otd_sha256d_search_vn<2, 0>(const otedama::Sha256dParamsV, VarPtr, uint32_t, uint64_t,
                                                       const otedama::HitSink);
template __global__ void otd_sha256d_search_vn<2, 5>(const otedama::Sha256dParamsV, VarPtr, uint32_t, uint64_t,
                                                       const otedama::HitSink);
template __global__ void otd_sha256d_search_vn<3, 0>(const otedama::Sha256dParamsV, VarPtr, uint32_t, uint64_t,
                                                       const otedama::HitSink);
template __global__ void otd_sha256d_search_vn<4, 0>(const otedama::Sha256dParamsV, VarPtr, uint32_t, uint64_t,
                                                       const otedama::HitSink);

namespace otedama {

hipError_t launch_sha256d_search_v(const Sha256dParamsV& p, const Sha256dVariant* vars, uint32_t base, uint64_t count,
                                   const HitSink& sink, int grid, hipStream_t stream, int block, int chains) {
  if (block != 64 && block != 256) return hipErrorInvalidValue;
  if (chains >= 2 && chains <= 4) {  // p.groups counts 64-variant groups; the kernel takes groups of 64 * chains
    if (p.groups == 0 || p.groups % uint32_t(chains) != 0) return hipErrorInvalidValue;
    Sha256dParamsV pn = p;
    pn.groups = p.groups / uint32_t(chains);
    if (grid <= 0 || (uint64_t(grid) * uint32_t(block / 64)) % pn.groups != 0) return hipErrorInvalidValue;
    const dim3 g(grid), b(block);
    if (chains == 2 && p.occupancy8)
      hipLaunchKernelGGL((otd_sha256d_search_vn<2, 5>), g, b, 0, stream, pn, vars, base, count, sink);
    else if (chains == 2)
      hipLaunchKernelGGL((otd_sha256d_search_vn<2, 0>), g, b, 0, stream, pn, vars, base, count, sink);
    else if (chains == 3)
      hipLaunchKernelGGL((otd_sha256d_search_vn<3, 0>), g, b, 0, stream, pn, vars, base, count, sink);
    else
      hipLaunchKernelGGL((otd_sha256d_search_vn<4, 0>), g, b, 0, stream, pn, vars, base, count, sink);
    return hipGetLastError();
  }
  if (chains != 1) return hipErrorInvalidValue;
  if (p.groups == 0 || grid <= 0 || (uint64_t(grid) * uint32_t(block / 64)) % p.groups != 0) return hipErrorInvalidValue;
  if (p.occupancy8)
    hipLaunchKernelGGL(otd_sha256d_search_v<8>, dim3(grid), dim3(block), 0, stream, p, vars, base, count, sink);
  else
    hipLaunchKernelGGL(otd_sha256d_search_v<0>, dim3(grid), dim3(block), 0, stream, p, vars, base, count, sink);
  return hipGetLastError();
}

}  // namespace otedama
