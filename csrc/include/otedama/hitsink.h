// Where a search kernel puts its hits, and how it learns that its batch is obsolete.
//
// Two consumers:
//  * the ops API (Python, torch-owned buffers): hits go to device memory, out[0] = count,
//    out[1 + words*i ...] = nonce (, variant); read back after the launch;
//  * the native GpuMiner: every hit is published the moment it is found into a ring of
//    HitRecords in host-coherent pinned memory (record, system-scope fence, then the tag),
//    and the miner thread consumes the ring while the launch is still running. The record
//    carries the low 32 bits of s_memrealtime (100 MHz) so the host can time the path from
//    the kernel's hit to the pool's accept.
// The abort word lives in uncached device memory (hipDeviceMallocUncached); the host bumps it
// when the work changes (a CPU store through the PCIe BAR, or hipStreamWriteValue32 on a control
// stream where the CPU cannot map it), and every wave checks it once per grid-stride iteration:
// a batch whose launch epoch is older stops early.
//
// Parity: the reference hands each share to the session the moment the worker finds it
// (internal/miner/worker.go:262-275) and switches work between 1024-nonce batches
// (worker.go:231-248); this is the same contract for launches of 10^8..10^9 nonces.
#pragma once
#include <cstdint>

namespace otedama {

struct HitRecord {
  uint32_t nonce;
  uint32_t variant;
  uint32_t stamp;  // s_memrealtime low 32 bits (100 MHz) at publication
  uint32_t tag;    // written last; equals the launch tag once the record is complete
};
static_assert(sizeof(HitRecord) == 16, "HitRecord is one 16-byte record");

struct HitSink {
  uint32_t* out = nullptr;          // out[0]: candidate count (device memory, atomicAdd)
  HitRecord* ring = nullptr;        // host-coherent records, or nullptr: legacy slots after out[0]
  const uint32_t* abort = nullptr;  // uncached device word; the batch stops once it is newer than `epoch`
  uint32_t cap = 0;                 // records / slots
  uint32_t tag = 0;                 // launch tag (never 0)
  uint32_t epoch = 0;               // launch epoch compared against *abort
  uint32_t words = 1;               // legacy slot width: 1 (nonce) or 2 (nonce, variant)
};

}  // namespace otedama
