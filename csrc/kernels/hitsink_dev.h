// Device side of otedama::HitSink (csrc/include/otedama/hitsink.h): hit publication and the abort poll.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "otedama/hitsink.h"

namespace otedama_dev {

// Abort word as of now (system-scope relaxed load: the word is uncached device memory the host stores to, through
// the BAR or a control stream). Wave-uniform by construction (one address), made provably so for a scalar branch. Without
// an abort word the batch's own epoch comes back, which never reads as newer.
__device__ __forceinline__ uint32_t abort_peek(const uint32_t* word, uint32_t epoch) {
  if (word == nullptr) return epoch;
  const uint32_t v = __hip_atomic_load(const_cast<uint32_t*>(word), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ uint32_t abort_peek(const otedama::HitSink& s) { return abort_peek(s.abort, s.epoch); }

// Split poll for loops: abort_issue starts the load and returns the raw (per-lane, equal) value; abort_seen, called
// one trip later, makes it wave-uniform and compares. abort_peek's readfirstlane right after the load makes the
// wave wait for an uncached system-scope load (~1-2 us) on every trip; split, the load's latency hides under the
// trip. (With 4 waves per SIMD the other waves covered most of that wait: the production miner measures the same
// with either form and the same as the tree before the abort word, within 0.2%, profiles/r3/u_miner_ab.)
__device__ __forceinline__ uint32_t abort_issue(const otedama::HitSink& s) {
  if (s.abort == nullptr) return s.epoch;
  return __hip_atomic_load(const_cast<uint32_t*>(s.abort), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Scalar-unit poll: one s_load from the word's (uniform) address straight into an SGPR, glc so it is served from
// memory and not from a stale scalar-cache line, and waited for in the same statement (the compiler does not track
// the counter of a load issued in asm). It holds no VGPR, so a loop at its VGPR budget (scrypt ROMix, 64) can poll
// without new spills. The wait also retires the wave's LDS operations in flight: place it where the loop waits for
// those anyway.
__device__ __forceinline__ uint32_t abort_peek_scalar(const otedama::HitSink& s) {
  if (s.abort == nullptr) return s.epoch;
  uint32_t v;
  asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(s.abort));
  return v;
}

// True once the host has moved the abort word past this batch's epoch (serial-number compare: wrap-safe).
__device__ __forceinline__ bool abort_newer(uint32_t word, uint32_t epoch) {
  return static_cast<int32_t>(word - epoch) > 0;
}
__device__ __forceinline__ bool abort_seen(uint32_t raw, uint32_t epoch) {
  return abort_newer(__builtin_amdgcn_readfirstlane(raw), epoch);
}

// One candidate. Miner path: the record is written, fenced at system scope, then tagged, so a host thread
// polling the tag never reads a half-written record. Ops path: the legacy device-memory slots.
__device__ __forceinline__ void hit_publish(const otedama::HitSink& s, uint32_t nonce, uint32_t variant) {
  const uint32_t slot = atomicAdd(s.out, 1u);
  if (slot >= s.cap) return;
  if (s.ring != nullptr) {
    otedama::HitRecord* r = s.ring + slot;
    r->nonce = nonce;
    r->variant = variant;
    r->stamp = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
    __threadfence_system();
    __hip_atomic_store(&r->tag, s.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else if (s.words == 2) {
    s.out[1 + 2 * slot] = nonce;
    s.out[2 + 2 * slot] = variant;
  } else {
    s.out[1 + slot] = nonce;
  }
}

}  // namespace otedama_dev
