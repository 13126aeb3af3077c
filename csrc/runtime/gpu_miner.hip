// GpuMiner: one host thread per GPU driving search batches on private HIP streams.
//
// Share path: a kernel publishes each hit the moment it is found into a ring of HitRecords in host-coherent
// pinned memory (record, system-scope fence, tag: otedama/hitsink.h). This thread polls the rings of the
// batches in flight every ~100 us, re-verifies each candidate on the CPU (full 256-bit compare against the
// job's current target) and pushes the share to the queue, whose eventfd wakes the control plane. A hit is
// therefore on its way to the pool while the launch that found it is still running, instead of after the
// batch (2^29 nonces, ~28 ms) and its copy-back.
//
// Job switches: new work opens a new launch epoch and writes it to an uncached device word. The CPU stores it
// straight into VRAM through the PCIe BAR when the runtime lets the CPU agent map the word; otherwise the store is a
// hipStreamWriteValue32 on a high-priority control stream, one more hardware queue (a 173 MiB host mapping,
// profiles/r4/c_host_abort/rss.jsonl). Every wave polls that word once per grid-stride trip, so batches of the old
// epoch stop within one trip (tens of us for SHA-256d, <= ~2 ms of ROMix for scrypt) and the first batch of the new
// work starts right behind them. The switch time (set_job -> new batch running) is recorded.
//
// Launch overlap: the two batches in flight sit on two streams (one per slot), so the next SHA-256d batch's waves
// fill the CUs that the running batch's tail leaves idle; without it a 2^29-nonce launch (28 ms) lost ~2.5% to its
// tail (profiles/r3/e_rehearsal). scrypt and X11 batches have per-slot buffers too (two 64 GiB halves of the scrypt
// pad, two X11 digest planes): the two scrypt half-batches run staggered by half a hash so that one of them reaches a
// ROMix phase boundary (its abort poll) every quarter hash, and a job switch waits ~T/8 instead of ~T/4 for the
// first half of the GPU to take the new work. OTEDAMA_SCRYPT_HALVES=0 / OTEDAMA_X11_OVERLAP=0 restore one shared
// buffer per algorithm with the batches chained (the A/B baselines).
//
// Device time: s_memrealtime (100 MHz) is mapped to CLOCK_MONOTONIC by a probe kernel at start-up (min round
// trip of several probes, before any search runs). After that every launch carries its own probe, queued on its
// stream just ahead of the search kernel: the host sees the stamp land while polling the hit rings, and each
// sighting bounds the offset from above (the store happened before it was seen). The mapping in use is the lowest
// bound of the last 2 s, so it follows drift between the two clocks without a stream or thread of its own, and a
// share carries the kernel's own hit time.
//
// Parity: the reference's worker sends each share as it is found (internal/miner/worker.go:262-275) and picks
// up new work between 1024-nonce batches (worker.go:231-248).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <unistd.h>

#include "otedama/clock_bounds.h"
#include "otedama/hitsink.h"
#include "otedama/job.h"
#include "otedama/runtime.h"
#include "otedama/sha256.h"
#include "otedama/trace.h"
#include "otedama/work_queue.h"
#include "otedama/x11_launch.h"

namespace otedama {

hipError_t launch_sha256d_search(const Sha256dParams& p, uint32_t base, uint64_t count, const HitSink& sink, int grid,
                                 hipStream_t stream);
hipError_t launch_sha256d_search_k(const Sha256dParamsK& p, uint32_t base, uint64_t count, const HitSink& sink,
                                   int grid, hipStream_t stream);
hipError_t launch_sha256d_search_v(const Sha256dParamsV& p, const Sha256dVariant* vars, uint32_t base, uint64_t count,
                                   const HitSink& sink, int grid, hipStream_t stream, int block = 256, int chains = 1);

hipError_t launch_scrypt_search(const ScryptParams& p, uint32_t base, uint32_t count, void* xbuf, void* scratch,
                                int gap, const HitSink& sink, int grid, hipStream_t stream);
uint64_t scrypt_scratch_bytes(int grid, int gap);
int gpu_cu_count(int device);

// Resident set of this process in MiB (/proc/self/statm), for the start-up phase record.
static double resident_mb() {
  FILE* f = std::fopen("/proc/self/statm", "r");
  if (!f) return 0;
  unsigned long size = 0, res = 0;
  const int n = std::fscanf(f, "%lu %lu", &size, &res);
  std::fclose(f);
  return n == 2 ? double(res) * double(sysconf(_SC_PAGESIZE)) / (1024.0 * 1024.0) : 0;
}

#define OTD_HIP(call)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (call);                                                                        \
    if (e_ != hipSuccess)                                                                          \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " #call); \
  } while (0)

}  // namespace otedama

// Device clock probe: one lane stores the 64-bit 100 MHz real-time counter (vector store to host memory).
__global__ void otd_rt_probe(uint64_t* out) {
  if (threadIdx.x == 0) *out = __builtin_amdgcn_s_memrealtime();
}

namespace otedama {

namespace {
// Hit-ring records per launch (16 B each, host-coherent). Launches are sized from the share target so the expected
// candidates per launch stay at or below kHitCap / 8 (see launch_cap); what still overflows is counted.
constexpr uint32_t kHitCap = 4096;
constexpr uint64_t kMinLaunchHashes = 1ull << 22;  // below ~0.2 ms per launch the launch overhead would dominate
constexpr size_t kVerifyCap = 8192;                // scrypt candidates waiting for host verification (~1 ms each)
constexpr int kInflight = 2;
constexpr double kRtHz = 100e6;
constexpr auto kIdlePoll = std::chrono::microseconds(100);
constexpr double kClockWindowS = 2.0;  // per-launch clock bounds kept for the device -> host mapping

// Let the CPU store to a device allocation directly: grant the CPU agent access (the allocation is VRAM, reachable
// through the PCIe BAR when the runtime exposes it) and confirm that the range is now mapped READ-WRITE in this process
// before anything touches it. libhsakmt reserves the GPU virtual-address range with PROT_NONE, so a mapping line alone
// proves nothing (small BAR, a VF without a mapped BAR): maps_range_writable requires the rw permissions. False leaves
// the word device-only (stores then go through a stream). The caller still verifies a store by reading it back.
bool cpu_store_map(void* p, size_t n) {
  hsa_agent_t cpu{};
  auto pick = [](hsa_agent_t a, void* data) -> hsa_status_t {
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
      *static_cast<hsa_agent_t*>(data) = a;
      return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
  };
  if (hsa_iterate_agents(pick, &cpu) != HSA_STATUS_INFO_BREAK) return false;
  if (hsa_amd_agents_allow_access(1, &cpu, nullptr, p) != HSA_STATUS_SUCCESS) return false;
  FILE* f = std::fopen("/proc/self/maps", "r");
  if (!f) return false;
  std::string maps;
  char buf[4096];
  size_t got;
  while ((got = std::fread(buf, 1, sizeof buf, f)) > 0) maps.append(buf, got);
  std::fclose(f);
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
  return maps_range_writable(maps, lo, lo + n);
}

// Header variants of one stripe group (up to 128 consecutive positions sharing block 2). Built once per
// (work generation, group) and shared by every launch of the group (~1000 launches at 2^29 nonces each).
struct Group {
  uint64_t gen = ~0ull, k = ~0ull;
  int nvar = 1;
  bool use_v = false;
  uint8_t header[kSha256dV2Group][80];
  uint32_t version[kSha256dV2Group] = {0}, ntime[kSha256dV2Group] = {0};
  uint64_t en2[kSha256dV2Group] = {0};
  Sha256dParamsV v_params{};
  Sha256dVariant v_table[kSha256dV2Group];
};

// A published hit handed to the verifier thread (scrypt), with everything needed to rebuild its header.
struct Candidate {
  std::shared_ptr<const JobTemplate> job;
  std::shared_ptr<const Group> group;
  uint64_t gen;
  uint32_t nonce, vi, stamp;
  double enq_host;
  uint32_t rt_enq;
  int nvar;
};

struct Batch {
  bool busy = false;
  std::shared_ptr<const JobTemplate> job;
  std::shared_ptr<const Group> group;
  uint64_t gen = 0;
  uint32_t epoch = 0, tag = 0;
  uint64_t count = 0;  // nonces per variant
  int nvar = 1;
  uint32_t consumed = 0;  // ring records already handled
  double enq_host = 0;    // monotonic seconds at enqueue
  uint32_t rt_enq = 0;    // device realtime (low 32 bits) estimated at enqueue
  bool started = false;
  hipStream_t stream = nullptr;  // this slot's stream
  hipEvent_t start{}, done{};
  uint32_t* d_count = nullptr;  // candidate counter (device memory)
  uint32_t* h_count = nullptr;  // pinned copy of the final count
  HitRecord* ring = nullptr;    // host-coherent records (host pointer)
  HitRecord* ring_dev = nullptr;  // the same records, device address
  Sha256dVariant* d_vars = nullptr;
  Sha256dVariant* h_vars = nullptr;
  uint64_t* h_clk = nullptr;  // this launch's clock probe (host-coherent; 0 until the probe ran)
  uint64_t* d_clk = nullptr;
  bool clk_pending = false;   // probe queued, its stamp not seen yet
  TraceId range = 0;
};
}  // namespace

GpuMiner::GpuMiner(int device, std::string device_id, uint64_t batch_nonces, int grid, size_t queue_cap, int sha_variants)
    : MinerBase(std::move(device_id), queue_cap), device_(device), batch_(batch_nonces), grid_(grid),
      sha_k_(sha_variants < 1 ? 1 : sha_variants > kSha256dMaxK ? kSha256dMaxK : sha_variants),
      sha_v_(sha_variants >= kSha256dVGroup), sha_v2_(sha_variants >= kSha256dV2Group) {
  if (batch_ == 0 || batch_ > (1ull << 32)) batch_ = 1ull << 30;
  // Batches must tile the 2^32 nonce range exactly.
  while ((1ull << 32) % batch_) --batch_;
}

GpuMiner::~GpuMiner() { stop(); }

void GpuMiner::start() {
  if (running_.exchange(true)) return;
  th_ = std::thread([this] {
    try {
      loop();
    } catch (const std::exception& ex) {
      // A device fault removes this device's stripe; the engine sees it in
      // stats().faulted and through the hashrate window.
      std::lock_guard<std::mutex> g(stats_mu_);
      stats_.faulted = true;
      stats_.error = ex.what();
    }
  });
}

void GpuMiner::stop() {
  if (!running_.exchange(false)) return;
  job_cv_.notify_all();
  if (th_.joinable()) th_.join();
}

void GpuMiner::loop() {
  trace_name_thread(("otedama-" + device_id_).c_str());
  double t_phase = monotonic_seconds();
  const double t_loop = t_phase;
  auto phase = [&](const char* name) {
    const double now = monotonic_seconds();
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.startup_ms.emplace_back(name, (now - t_phase) * 1e3);
    stats_.startup_rss_mb.emplace_back(name, resident_mb());
    t_phase = now;
  };
  OTD_HIP(hipSetDevice(device_));
  OTD_HIP(hipFree(nullptr));  // force runtime / context creation here so the phase below is honest
  phase("hip_set_device");
  hipStream_t ctl = nullptr;      // control stream: only when the CPU cannot store the abort word itself
  bool host_abort = false;       // the CPU stores the abort word through the BAR
  Batch slots[kInflight];
  uint32_t* d_abort = nullptr;   // uncached device word: the newest launch epoch that must keep running
  hipEvent_t ref_ev = nullptr;   // device-timeline origin of hashes_done_at_s
  uint64_t* h_rt = nullptr;      // probe outputs (pinned, host-coherent): start-up probe, then one line per slot
  uint64_t* d_rt = nullptr;      // their device address
  void* scratch = nullptr;       // scrypt pad, allocated on the first scrypt job (one half per slot)
  void* xbuf = nullptr;
  uint64_t* x11_h = nullptr;     // X11 intermediate digests (8 u64 planes x batch, one set per slot)
  // Released on every exit, including a HIP error thrown mid-loop (device fault): in-flight batches are drained
  // first so nothing is freed under a running kernel or copy.
  struct Release {
    std::function<void()> f;
    ~Release() { f(); }
  } release{[&] {
    for (auto& s : slots)
      if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (ctl) (void)hipStreamSynchronize(ctl);
    for (auto& s : slots) {
      if (s.d_count) (void)hipFree(s.d_count);
      if (s.h_count) (void)hipHostFree(s.h_count);
      if (s.ring) (void)hipHostFree(s.ring);
      if (s.start) (void)hipEventDestroy(s.start);
      if (s.done) (void)hipEventDestroy(s.done);
      if (s.d_vars) (void)hipFree(s.d_vars);
      if (s.h_vars) (void)hipHostFree(s.h_vars);
    }
    if (d_abort) (void)hipFree(d_abort);
    if (ref_ev) (void)hipEventDestroy(ref_ev);
    if (h_rt) (void)hipHostFree(h_rt);
    if (scratch) (void)hipFree(scratch);
    if (xbuf) (void)hipFree(xbuf);
    if (x11_h) (void)hipFree(x11_h);
    for (auto& s : slots)
      if (s.stream && (&s == &slots[0] || s.stream != slots[0].stream)) (void)hipStreamDestroy(s.stream);
    if (ctl) (void)hipStreamDestroy(ctl);
  }};
  // Search streams: one per in-flight batch, so a launch's tail overlaps the next launch's first waves; with
  // OTEDAMA_SEARCH_STREAMS=1 the batches share one stream (one hardware queue less, 173 MiB of host memory).
  const char* ss_env = std::getenv("OTEDAMA_SEARCH_STREAMS");
  const bool one_stream = ss_env && std::atoi(ss_env) == 1;
  // OTEDAMA_RESERVE_CUS=<cu>,<cu>,...: the search streams get a CU mask without these CUs, so a kernel of another
  // process on the same GPU (a node rank's RCCL collective) finds a free slot at once instead of waiting for a
  // mining workgroup to finish (parallel/comm_probe.py measures the trade: the reserved CUs' share of the rate).
  std::vector<uint32_t> cu_mask;
  int reserved = 0;
  if (const char* rc_env = std::getenv("OTEDAMA_RESERVE_CUS")) {
    const int ncu = gpu_cu_count(device_) > 0 ? gpu_cu_count(device_) : 256;
    cu_mask.assign((ncu + 31) / 32, 0xFFFFFFFFu);
    if (ncu % 32) cu_mask.back() = (1u << (ncu % 32)) - 1u;
    for (const char* q = rc_env; *q;) {
      char* end = nullptr;
      const long cu = std::strtol(q, &end, 10);
      if (end == q) break;
      if (cu >= 0 && cu < ncu && (cu_mask[cu / 32] >> (cu % 32) & 1u)) {
        cu_mask[cu / 32] &= ~(1u << (cu % 32));
        ++reserved;
      }
      q = (*end == ',') ? end + 1 : end;
    }
  }
  for (int i = 0; i < kInflight; ++i) {
    if (one_stream && i > 0) slots[i].stream = slots[0].stream;
    else if (reserved > 0)
      OTD_HIP(hipExtStreamCreateWithCUMask(&slots[i].stream, uint32_t(cu_mask.size()), cu_mask.data()));
    else OTD_HIP(hipStreamCreateWithFlags(&slots[i].stream, hipStreamNonBlocking));
  }
  {
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.reserved_cus = uint64_t(reserved);
  }
  // The abort word must never wait behind a search kernel. The CPU stores it itself when it can map the word
  // (OTEDAMA_HOST_ABORT=0 forces the stream form). Otherwise the store goes on a high-priority stream: HIP
  // multiplexes streams of one priority onto GPU_MAX_HW_QUEUES (4) hardware queues, and with two search streams
  // plus torch's in the same process a control stream can land on a busy queue, where its write waits for a whole
  // 2^32-hash launch (the job switch grew from 0.3 ms to ~110 ms); high-priority streams come from a separate pool.
  // Every hardware queue costs a 173 MiB host mapping (tools/queue_rss.hip, profiles/r4/c_host_abort/rss.jsonl).
  OTD_HIP(hipExtMallocWithFlags(reinterpret_cast<void**>(&d_abort), 256, hipDeviceMallocUncached));
  // on a search stream: the first use of the null stream would give this process one more hardware queue
  // (tools/queue_rss.hip, profiles/r4/d_queues)
  OTD_HIP(hipMemsetAsync(d_abort, 0, 256, slots[0].stream));
  OTD_HIP(hipStreamSynchronize(slots[0].stream));
  const char* ha_env = std::getenv("OTEDAMA_HOST_ABORT");
  host_abort = !(ha_env && ha_env[0] == '0') && cpu_store_map(d_abort, 256);
  if (host_abort) {
    // Prove the path before trusting it: a CPU store must land in VRAM where the device (a copy on a search stream)
    // reads it back. Anything else (a mapping that swallows writes) falls back to the control stream.
    for (uint32_t probe : {0xA5C3E10Fu, 0u}) {
      __atomic_store_n(d_abort, probe, __ATOMIC_RELEASE);
      _mm_sfence();
      uint32_t back = ~probe;
      OTD_HIP(hipMemcpyAsync(&back, d_abort, sizeof back, hipMemcpyDeviceToHost, slots[0].stream));
      OTD_HIP(hipStreamSynchronize(slots[0].stream));
      if (back != probe) { host_abort = false; break; }
    }
    if (!host_abort) {  // the word must read 0 whichever path stores it from now on
      OTD_HIP(hipMemsetAsync(d_abort, 0, 256, slots[0].stream));
      OTD_HIP(hipStreamSynchronize(slots[0].stream));
    }
  }
  if (!host_abort) {
    int prio_lo = 0, prio_hi = 0;
    OTD_HIP(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    OTD_HIP(hipStreamCreateWithPriority(&ctl, hipStreamNonBlocking, prio_hi));
  }
  {
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.host_abort = host_abort;
  }
  phase("streams");
  OTD_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_rt), 64 * (1 + kInflight), hipHostMallocCoherent | hipHostMallocMapped));
  std::memset(h_rt, 0, 64 * (1 + kInflight));
  OTD_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_rt), h_rt, 0));
  for (int i = 0; i < kInflight; ++i) {
    slots[i].h_clk = h_rt + 8 * (1 + i);
    slots[i].d_clk = d_rt + 8 * (1 + i);
  }
  phase("control_words");
  for (auto& s : slots) {
    OTD_HIP(hipMalloc(&s.d_count, 64));
    OTD_HIP(hipHostMalloc(reinterpret_cast<void**>(&s.h_count), 64, hipHostMallocDefault));
    OTD_HIP(hipHostMalloc(reinterpret_cast<void**>(&s.ring), kHitCap * sizeof(HitRecord),
                          hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(s.ring, 0, kHitCap * sizeof(HitRecord));
    OTD_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&s.ring_dev), s.ring, 0));
    OTD_HIP(hipEventCreate(&s.start));
    OTD_HIP(hipEventCreate(&s.done));
    if (sha_v_) {
      OTD_HIP(hipMalloc(&s.d_vars, kSha256dV2Group * sizeof(Sha256dVariant)));
      OTD_HIP(hipHostMalloc(&s.h_vars, kSha256dV2Group * sizeof(Sha256dVariant), hipHostMallocDefault));
    }
  }
  phase("buffers");
  const int cus = gpu_cu_count(device_) > 0 ? gpu_cu_count(device_) : 256;
  // Lane-cooperative full-line ROMix (gap 1, nt pad traffic, 16 blocks/CU = 128 GiB of HBM): ~16.75 MH/s vs
  // 13.6-14.0 for the per-lane kernels at gap 1/2 (profiles/r1/scrypt_romix_ab.md).
  const int scrypt_gap = kScryptCoop;
  const int scrypt_grid = cus * 16;
  const uint32_t scrypt_batch = uint32_t(scrypt_grid) * 256u;
  const char* halves_env = std::getenv("OTEDAMA_SCRYPT_HALVES");
  const bool scrypt_halves = !(halves_env && halves_env[0] == '0');
  const char* x11ov_env = std::getenv("OTEDAMA_X11_OVERLAP");
  const bool x11_overlap = !(x11ov_env && x11ov_env[0] == '0');
  double scrypt_hash_s = 0.064;  // one lane's scrypt hash (= one full batch) on the device; refined per batch
  // X11: eleven stage kernels per batch over a 64 B/nonce digest buffer (512 MiB at 2^23).
  const uint32_t x11_batch = 1u << 23;
  // K-variant SHA-256d kernel: 16 blocks of 256 per CU (tools/bench_sha_k.py, profiles/r2/).
  grid_k_ = cus * 16;
  // Version-parallel kernel (8-waves/SIMD build): 64 blocks of 256 per CU (profiles/r2/sha_v).
  grid_v_ = cus * 64;
  // Two-chain kernel (4 waves/SIMD build): 128 blocks of 256 per CU (profiles/r2/sha_v2).
  grid_v2_ = cus * 128;

  // ---- device clock -> host clock
  std::atomic<double> rt_offset{0.0};  // host monotonic seconds at device realtime 0
  double calib_rtt = 1e9;
  // Start-up: probes bracketed by the launch and the stream sync on an idle device; the tightest bracket wins.
  auto probe = [&](hipStream_t on) {
    __atomic_store_n(h_rt, 0ull, __ATOMIC_RELEASE);
    const double t0 = monotonic_seconds();
    hipLaunchKernelGGL(otd_rt_probe, dim3(1), dim3(64), 0, on, d_rt);
    OTD_HIP(hipGetLastError());
    OTD_HIP(hipStreamSynchronize(on));
    const double t1 = monotonic_seconds();
    const uint64_t rt = __atomic_load_n(h_rt, __ATOMIC_ACQUIRE);
    if (rt && (t1 - t0) < calib_rtt) {
      rt_offset.store(0.5 * (t0 + t1) - double(rt) / kRtHz);
      calib_rtt = t1 - t0;
      std::lock_guard<std::mutex> g(stats_mu_);
      stats_.clock_calib_rtt_us = (t1 - t0) * 1e6;
    }
  };
  for (int t = 0; t < 8; ++t) probe(slots[0].stream);
  rt_offset_ = rt_offset.load();
  phase("clock_calibration");
  OTD_HIP(hipEventCreate(&ref_ev));
  OTD_HIP(hipEventRecord(ref_ev, slots[0].stream));  // before any search: the device-timeline origin
  bool first_switch = true;
  // Running: every launch's probe gives an upper bound on the offset (host time it was seen minus its device
  // time); the lowest bound of the last kClockWindowS seconds is the mapping in use.
  ClockBounds clk_bounds(kClockWindowS);
  auto clock_seen = [&](Batch& b) {
    const uint64_t rt = __atomic_load_n(b.h_clk, __ATOMIC_ACQUIRE);
    if (!rt) return;
    const double now = monotonic_seconds();  // after the load that saw the stamp: a valid upper bound
    b.clk_pending = false;
    rt_offset.store(clk_bounds.add(now, now - double(rt) / kRtHz));
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.clock_samples += 1;
  };
  auto write_abort = [&](uint32_t e) {
    if (host_abort) {
      __atomic_store_n(d_abort, e, __ATOMIC_RELEASE);
      _mm_sfence();  // out of the write-combining buffers and onto the bus now
    } else {
      OTD_HIP(hipStreamWriteValue32(ctl, d_abort, e, 0));
    }
  };

  std::shared_ptr<Group> group;  // current stripe group
  uint64_t cur_gen = ~0ull;
  uint64_t k = 0;  // variant-stripe position of the current group
  uint64_t nonce_off = 0;
  uint32_t epoch = 1, tag = 0;
  uint64_t epoch_gen = ~0ull;  // work generation the current epoch was opened for (0 = paused)
  bool switch_pending = false;
  double switch_t0 = 0;
  double rate_hpms = 0;  // hashes per ms of completed full batches (for aborted-batch accounting)
  std::deque<int> fifo;  // in-flight slots, issue order
  BoundedWorkQueue<Candidate> vq(kVerifyCap);  // scrypt candidates awaiting host verification
  std::thread verifier;

  // New work opens a new launch epoch and moves the device abort word: batches of older epochs stop at
  // their next poll. Called at the top of every loop trip and between hit verifications (a burst of scrypt hits
  // costs ~1 ms of CPU each and must not delay a switch).
  auto check_epoch = [&](uint64_t* gen_out) {
    uint64_t gen = 0;
    double set_at = 0;
    auto job = peek_job(&gen, &set_at);
    // A pause (no job) keeps the batches in flight running to their end (<= kInflight launches): moving the abort
    // word for it would skip the unsearched rest of those batches for good when the same work resumes, since the
    // cursor already moved past them. Only new work stops them.
    const uint64_t want_gen = job ? gen : epoch_gen;
    if (want_gen != epoch_gen) {
      epoch_gen = want_gen;
      ++epoch;
      if (!fifo.empty()) write_abort(epoch);
      if (job) { switch_pending = true; switch_t0 = set_at; }
    }
    if (gen_out) *gen_out = gen;
    return job;
  };

  auto verify_push = [&](const Candidate& b, uint32_t nonce, uint32_t vi, uint32_t stamp, bool stamped,
                         const std::shared_ptr<const JobTemplate>& cur, uint64_t cur_g, uint64_t* good,
                         uint64_t* bad, const uint8_t* pre_hash = nullptr) {
    if (vi >= (uint32_t)b.nvar) { ++*bad; return; }
    uint8_t hdr[80];
    std::memcpy(hdr, b.group->header[vi], 80);
    store_le32(hdr + 76, nonce);
    ShareRecord r{};
    // A target-only update (same work generation) applies to batches in flight too: their hits are checked
    // against, and reported under, the current template (its target and control-plane epoch).
    const JobTemplate* tj = (cur && cur_g == b.gen) ? cur.get() : b.job.get();
    if (pre_hash) {
      std::memcpy(r.hash, pre_hash, 32);
      if (!le256_leq(r.hash, tj->target)) { ++*bad; return; }
    } else if (!verify_share(b.job->algo, hdr, tj->target, r.hash)) {
      ++*bad;
      return;
    }
    r.epoch = tj->epoch; r.job_id = tj->job_id; r.channel_id = tj->channel_id;
    r.nonce = nonce; r.ntime = b.group->ntime[vi]; r.version = b.group->version[vi]; r.extranonce2 = b.group->en2[vi];
    r.extranonce2_size = b.job->extranonce2_size; r.device_id = device_id_;
    r.found_at = monotonic_seconds();
    if (stamped) r.device_found_at = b.enq_host + double(int32_t(stamp - b.rt_enq)) / kRtHz;
    queue_.push(std::move(r));
    ++*good;
  };

  // Scrypt candidates are re-hashed up to sixteen at a time (AVX-512 lanes, ~4x the scalar rate per hash; AVX2
  // passes of eight without it), so a burst of easy-target hits drains in a fraction of the time.
  verifier = std::thread([&] {
    std::vector<Candidate> cs;
    cs.reserve(16);
    uint8_t hb[16][80], ho[16][32];
    const uint8_t* ip[16];
    uint8_t* op[16];
    for (int l = 0; l < 16; ++l) { ip[l] = hb[l]; op[l] = ho[l]; }
    while (cs.clear(), vq.pop_many(&cs, 16) > 0) {  // 0 once stopped and drained
      uint64_t good = 0, bad = 0, g = 0;
      auto cur = peek_job(&g, nullptr);
      int n = 0;
      for (const Candidate& c : cs) {
        if (c.job->algo != Algo::kScrypt || c.vi >= (uint32_t)c.nvar) continue;
        std::memcpy(hb[n], c.group->header[c.vi], 80);
        store_le32(hb[n] + 76, c.nonce);
        ++n;
      }
      if (n > 0) scrypt_1024_1_1_batch(n, ip, op);
      int l = 0;
      for (const Candidate& c : cs) {
        const bool batched = c.job->algo == Algo::kScrypt && c.vi < (uint32_t)c.nvar;
        verify_push(c, c.nonce, c.vi, c.stamp, true, cur, g, &good, &bad, batched ? ho[l] : nullptr);
        l += batched;
      }
      std::lock_guard<std::mutex> sg(stats_mu_);
      stats_.shares += good;
      stats_.rejected_candidates += bad;
    }
  });
  struct VerifierJoin {
    std::function<void()> f;
    ~VerifierJoin() { f(); }
  } verifier_join{[&] {
    vq.stop(running_.load() ? ~size_t(0) : 64);  // shutting down: bound the work left (~1 ms each)
    if (verifier.joinable()) verifier.join();
  }};

  // Consume the published records of a batch; `final_n` = the batch's final count (after completion) or ~0u
  // while it runs. Returns the number of records handled.
  auto drain_ring = [&](Batch& b, uint32_t final_n, const std::shared_ptr<const JobTemplate>& cur,
                        uint64_t cur_g) -> uint32_t {
    const uint32_t limit = final_n == ~0u ? kHitCap : std::min(final_n, kHitCap);
    uint64_t good = 0, bad = 0, lost = 0, handled = 0;
    while (b.consumed < limit) {
      HitRecord* r = b.ring + b.consumed;
      const uint32_t tg = __atomic_load_n(&r->tag, __ATOMIC_ACQUIRE);
      if (tg != b.tag) {
        if (final_n == ~0u) break;  // not written yet
        ++lost;                     // completed launch without its record: count and skip (should not happen)
        ++b.consumed;
        continue;
      }
      const uint32_t nonce = __atomic_load_n(&r->nonce, __ATOMIC_RELAXED);
      const uint32_t vi = __atomic_load_n(&r->variant, __ATOMIC_RELAXED);
      const uint32_t stamp = __atomic_load_n(&r->stamp, __ATOMIC_RELAXED);
      if (b.job->algo == Algo::kScrypt) {
        // host scrypt costs ~1 ms per candidate: verified on the verifier thread so a burst of candidates never
        // holds up a job switch or the next launch. The queue is bounded: past kVerifyCap a candidate is refused
        // and counted (a share target far below the device's rate would otherwise grow it without limit).
        vq.push(Candidate{b.job, b.group, b.gen, nonce, vi, stamp, b.enq_host, b.rt_enq, b.nvar});
      } else {
        verify_push(Candidate{b.job, b.group, b.gen, 0, 0, 0, b.enq_host, b.rt_enq, b.nvar}, nonce, vi, stamp, true,
                    cur, cur_g, &good, &bad);
      }
      ++b.consumed;
      ++handled;
    }
    if (handled || lost) {
      const uint64_t refused = vq.refused(), peak = vq.peak();
      std::lock_guard<std::mutex> g(stats_mu_);
      stats_.shares += good;
      stats_.rejected_candidates += bad + lost;
      if (final_n == ~0u) stats_.ring_hits += handled;
      stats_.verify_dropped = refused;
      stats_.verify_queue_peak = peak;
    }
    return uint32_t(handled);
  };

  auto finish = [&](Batch& b, const std::shared_ptr<const JobTemplate>& cur, uint64_t cur_g) {
    trace_stop(b.range);
    const uint32_t n = *b.h_count;
    drain_ring(b, n, cur, cur_g);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, b.start, b.done);
    float done_ms = 0;  // device-timeline completion of this batch, for exact-window hash rates
    const bool have_done = hipEventElapsedTime(&done_ms, ref_ev, b.done) == hipSuccess;
    const uint64_t full = b.count * uint64_t(b.nvar);
    const bool aborted = int32_t(epoch - b.epoch) > 0;  // a newer epoch was opened after this batch
    uint64_t done_hashes = full;
    if (aborted && rate_hpms > 0) done_hashes = std::min<uint64_t>(full, uint64_t(rate_hpms * double(ms)));
    if (!aborted && ms > 0) rate_hpms = rate_hpms > 0 ? 0.8 * rate_hpms + 0.2 * (double(full) / ms) : double(full) / ms;
    if (!aborted && ms > 0 && b.job && b.job->algo == Algo::kScrypt) scrypt_hash_s = 0.7 * scrypt_hash_s + 0.3e-3 * ms;
    std::lock_guard<std::mutex> g(stats_mu_);
    if (n > kHitCap) {  // the kernel counted these candidates but had no ring slot left to publish them
      if (stats_.ring_overflow == 0)
        std::fprintf(stderr, "otedama: %s: launch found %u candidates, hit ring holds %u: %u lost (counted in "
                     "ring_overflow)\n", device_id_.c_str(), n, kHitCap, n - kHitCap);
      stats_.ring_overflow += n - kHitCap;
    }
    stats_.hashes += done_hashes;
    if (have_done) stats_.hashes_done_at_s = std::max(stats_.hashes_done_at_s, double(done_ms) * 1e-3);
    stats_.candidates += n;
    stats_.busy_seconds += ms * 1e-3;
    stats_.launches += 1;
    if (aborted) stats_.aborted_launches += 1;
    if (b.nvar > 1) stats_.variant_launches += 1;
    b.busy = false;
    b.job.reset();
    b.group.reset();
  };

  auto build_group = [&](const std::shared_ptr<const JobTemplate>& job, uint64_t gen) {
    auto gp = std::make_shared<Group>();
    gp->gen = gen;
    gp->k = k;
    gp->nvar = 1;
    const uint64_t v = job->variant_start + k * job->variant_stride;
    job->variant_header(v, gp->header[0], &gp->version[0], &gp->ntime[0], &gp->en2[0]);
    if (job->algo == Algo::kSha256d && (sha_v_ || sha_k_ > 1)) {
      // Consecutive stripe positions whose headers differ only in block 1 (version rolling) share block 2: up to
      // 128 (two-chain version-parallel kernel), 64 (one chain) or K (per-lane K-variant kernel). A group is
      // all-or-nothing per layout and depends only on (work, k), so all its launches use one kernel.
      const int want = sha_v2_ ? kSha256dV2Group : sha_v_ ? kSha256dVGroup : sha_k_;
      int kv = 1;
      while (kv < want) {
        const uint64_t vk = job->variant_start + (k + kv) * job->variant_stride;
        if (vk >= job->variant_space()) break;
        job->variant_header(vk, gp->header[kv], &gp->version[kv], &gp->ntime[kv], &gp->en2[kv]);
        if (std::memcmp(gp->header[kv] + 64, gp->header[0] + 64, 12) != 0) break;
        ++kv;
      }
      if (sha_v2_ && kv >= kSha256dV2Group) {
        gp->use_v = true;
        gp->nvar = kSha256dV2Group;
      } else if (sha_v_ && kv >= kSha256dVGroup) {
        gp->use_v = true;
        gp->nvar = kSha256dVGroup;
      } else if (sha_k_ > 1) {
        gp->nvar = sha256d_k_floor(std::min(kv, sha_k_));  // kernels exist for K in {2,3,4,6,8,12,16}
      }
      if (gp->use_v) {
        const uint8_t* hs[kSha256dV2Group];
        for (int j = 0; j < gp->nvar; ++j) hs[j] = gp->header[j];
        if (!sha256d_prepare_v(hs, gp->nvar, job->target, &gp->v_params, gp->v_table))
          throw std::runtime_error("sha256d_prepare_v");
        gp->v_params.occupancy8 = gp->nvar == kSha256dV2Group ? 0 : 1;
      }
    }
    return gp;
  };

  // Hashes per launch for a share target: the kernels' prefilter passes a hash whose top word is <= the target's,
  // i.e. with probability (target_hi + 1) / 2^32, so expected candidates per launch = hashes * that. Launches are cut
  // (powers of two, so they still tile 2^32) until that is <= kHitCap / 8; the hit ring then overflows only on a
  // draw ~8 sigma above the mean at the floor target, and any overflow is counted.
  const char* cap_env = std::getenv("OTEDAMA_LAUNCH_CAP");  // "0": launches keep batch_ hashes (overflow tests)
  const bool cap_launches = !(cap_env && cap_env[0] == '0');
  auto launch_cap = [&](const JobTemplate& job) -> uint64_t {
    if (!cap_launches) return 1ull << 40;
    const double p = (double(load_le32(job.target + 28)) + 1.0) / 4294967296.0;
    const double lim = double(kHitCap / 8) / p;
    uint64_t cap = 1ull << 40;
    while (cap > kMinLaunchHashes && double(cap) > lim) cap >>= 1;
    return cap;
  };

  auto enqueue = [&](Batch& s, const std::shared_ptr<const JobTemplate>& job, uint64_t gen, const Batch* prev) {
    hipStream_t stream = s.stream;
    if (!group || group->gen != gen || group->k != k) group = build_group(job, gen);
    s.job = job;
    s.group = group;
    s.gen = gen;
    s.nvar = group->nvar;
    s.epoch = epoch;
    s.tag = ++tag == 0 ? ++tag : tag;
    s.consumed = 0;
    s.started = false;
    s.range = trace_start(job->algo == Algo::kScrypt ? "otd.scrypt.batch"
                          : job->algo == Algo::kX11  ? "otd.x11.batch"
                                                     : "otd.sha256d.batch");
    HitSink sink;
    sink.out = s.d_count;
    sink.ring = s.ring_dev;
    sink.abort = d_abort;
    sink.cap = kHitCap;
    sink.tag = s.tag;
    sink.epoch = s.epoch;
    sink.words = 2;
    // scrypt pad / X11 digests are shared by the batches: chain them; SHA-256d batches overlap freely
    const bool shared_buf = (job->algo == Algo::kScrypt && !scrypt_halves) || (job->algo == Algo::kX11 && !x11_overlap);
    if (prev && prev->busy && shared_buf) OTD_HIP(hipStreamWaitEvent(stream, prev->done, 0));
    const int slot_i = int(&s - slots);
    OTD_HIP(hipMemsetAsync(s.d_count, 0, 64, stream));
    OTD_HIP(hipEventRecord(s.start, stream));
    __atomic_store_n(s.h_clk, 0ull, __ATOMIC_RELEASE);
    hipLaunchKernelGGL(otd_rt_probe, dim3(1), dim3(64), 0, stream, s.d_clk);
    OTD_HIP(hipGetLastError());
    s.clk_pending = true;
    s.enq_host = monotonic_seconds();
    rt_offset_ = rt_offset.load();
    s.rt_enq = uint32_t(uint64_t((s.enq_host - rt_offset_) * kRtHz));
    if (job->algo == Algo::kScrypt) {
      if (!scratch) {
        OTD_HIP(hipMalloc(&scratch, scrypt_scratch_bytes(scrypt_grid, scrypt_gap)));
        OTD_HIP(hipMalloc(&xbuf, uint64_t(scrypt_batch) * 128));
      }
      ScryptParams p;
      scrypt_prepare(group->header[0], job->target, &p);
      const uint64_t remaining = (1ull << 32) - nonce_off;
      // halves: each slot owns half the pad / X buffer and half the grid (the two run side by side)
      const int grid = scrypt_halves ? scrypt_grid / 2 : scrypt_grid;
      const uint32_t lanes = scrypt_halves ? scrypt_batch / 2 : scrypt_batch;
      char* pad = static_cast<char*>(scratch) +
                  (scrypt_halves ? uint64_t(slot_i) * scrypt_scratch_bytes(grid, scrypt_gap) : 0);
      char* xb = static_cast<char*>(xbuf) + (scrypt_halves ? uint64_t(slot_i) * lanes * 128ull : 0);
      s.count = std::min<uint64_t>({remaining, lanes, launch_cap(*job)});
      OTD_HIP(launch_scrypt_search(p, uint32_t(nonce_off), uint32_t(s.count), xb, pad, scrypt_gap, sink, grid,
                                   stream));
    } else if (job->algo == Algo::kX11) {
      if (!x11_h) OTD_HIP(hipMalloc(&x11_h, uint64_t(x11_batch) * 64 * (x11_overlap ? kInflight : 1)));
      X11Params p;
      x11_prepare(group->header[0], job->target, &p);
      const uint64_t remaining = (1ull << 32) - nonce_off;
      s.count = std::min<uint64_t>({remaining, x11_batch, launch_cap(*job)});
      uint64_t* H = x11_h + (x11_overlap ? uint64_t(slot_i) * x11_batch * 8 : 0);
      OTD_HIP(x11_launch_chain(p, uint32_t(nonce_off), H, x11_batch, uint32_t(s.count), &sink, stream));
    } else if (group->use_v) {
      const bool two = group->nvar == kSha256dV2Group;
      Sha256dParamsV vp = group->v_params;
      // The table is cached per (work, group) but a target-only update (SV2 SetTarget, V1 set_difficulty) keeps
      // the work generation: the share filter follows the job's current target on every launch.
      vp.target_hi = load_le32(job->target + 28);
      const size_t table_bytes = size_t(group->nvar) * sizeof(Sha256dVariant);
      std::memcpy(s.h_vars, group->v_table, table_bytes);
      OTD_HIP(hipMemcpyAsync(s.d_vars, s.h_vars, table_bytes, hipMemcpyHostToDevice, stream));
      // W3 (big-endian nonce word) windows tile [0, 2^32) exactly like the nonce windows of the other kernels;
      // the kernel reports nonce = bswap(W3). Launch duration stays batch_ hashes.
      const uint64_t launch = std::min(batch_, launch_cap(*job));
      s.count = std::min<uint64_t>(launch >= uint64_t(group->nvar) ? launch / uint64_t(group->nvar) : 1,
                                   (1ull << 32) - nonce_off);
      OTD_HIP(launch_sha256d_search_v(vp, s.d_vars, uint32_t(nonce_off), s.count, sink, two ? grid_v2_ : grid_v_,
                                      stream, 256, two ? 2 : 1));
    } else if (group->nvar > 1) {
      Sha256dParamsK p;
      const uint8_t* hs[kSha256dMaxK];
      for (int j = 0; j < group->nvar; ++j) hs[j] = group->header[j];
      if (!sha256d_prepare_k(hs, group->nvar, job->target, &p)) throw std::runtime_error("sha256d_prepare_k");
      // Keep one launch's duration about independent of K: nonces per variant = batch / (largest power of two
      // <= K); batch is a power of two that tiles 2^32, so this still tiles it.
      const uint64_t launch = std::min(batch_, launch_cap(*job));
      uint64_t div = 1;
      while (div * 2 <= (uint64_t)group->nvar && div * 2 <= launch) div *= 2;
      s.count = std::min<uint64_t>(launch / div, (1ull << 32) - nonce_off);
      OTD_HIP(launch_sha256d_search_k(p, uint32_t(nonce_off), s.count, sink, grid_k_, stream));
    } else {
      Sha256dParams p;
      sha256d_prepare(group->header[0], job->target, &p);
      s.count = std::min<uint64_t>(std::min(batch_, launch_cap(*job)), (1ull << 32) - nonce_off);
      OTD_HIP(launch_sha256d_search(p, uint32_t(nonce_off), s.count, sink, grid_, stream));
    }
    OTD_HIP(hipMemcpyAsync(s.h_count, s.d_count, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    OTD_HIP(hipEventRecord(s.done, stream));
    s.busy = true;
    nonce_off += s.count;
    const uint64_t launch_hashes = s.count * uint64_t(s.nvar);
    const uint64_t group_n = uint64_t(group->nvar);
    if (nonce_off >= (1ull << 32)) { nonce_off = 0; k += group_n; }
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.variant_epoch = job->epoch;
    stats_.launch_hashes = launch_hashes;
    stats_.variant_next = job->variant_start + (nonce_off == 0 ? k : k + group_n) * job->variant_stride;
  };

  while (running_.load()) {
    uint64_t gen = 0;
    auto job = check_epoch(&gen);
    bool progressed = false;
    if (job && gen != cur_gen) { cur_gen = gen; k = 0; nonce_off = 0; }
    // 1) hits of the batches in flight, oldest first, and the clock stamps of launches that just started
    for (int i : fifo)
      if (slots[i].clk_pending) clock_seen(slots[i]);
    for (int i : fifo) progressed |= drain_ring(slots[i], ~0u, job, gen) > 0;
    // 2) retire completed batches (the two streams may complete out of issue order)
    for (auto it = fifo.begin(); it != fifo.end();) {
      Batch& b = slots[*it];
      const hipError_t q = hipEventQuery(b.done);
      if (q == hipErrorNotReady) { ++it; continue; }
      OTD_HIP(q);
      if (!b.started) b.started = true;
      finish(b, job, gen);
      it = fifo.erase(it);
      progressed = true;
    }
    // 3) job-switch time: set_job -> the first batch of the new epoch running on the device
    if (switch_pending) {
      for (int i : fifo) {
        Batch& b = slots[i];
        if (b.epoch != epoch) continue;
        const hipError_t q = hipEventQuery(b.start);
        if (q == hipErrorNotReady) break;
        OTD_HIP(q);
        b.started = true;
        const double ms = (monotonic_seconds() - switch_t0) * 1e3;
        switch_pending = false;
        std::lock_guard<std::mutex> g(stats_mu_);
        if (first_switch) {
          first_switch = false;
          double before = 0;  // the phases above, so the wait is what is left of loop start -> set_job
          for (const auto& kv : stats_.startup_ms) before += kv.second;
          stats_.startup_ms.emplace_back("wait_first_job", std::max(0.0, (switch_t0 - t_loop) * 1e3 - before));
          stats_.startup_ms.emplace_back("first_batch", ms);
        }
        stats_.job_switches += 1;
        stats_.last_job_switch_ms = ms;
        stats_.job_switch_ms.push_back(ms);
        if (stats_.job_switch_ms.size() > 64) stats_.job_switch_ms.erase(stats_.job_switch_ms.begin());
        stats_.work_started.emplace_back(job ? job->epoch : 0, switch_t0 + ms * 1e-3);
        if (stats_.work_started.size() > 64) stats_.work_started.erase(stats_.work_started.begin());
        break;
      }
    }
    // 4) keep kInflight batches queued
    while (job && (int)fifo.size() < kInflight) {
      const uint64_t v = job->variant_start + k * job->variant_stride;
      if (v >= job->variant_space()) break;  // stripe exhausted: wait for fresh work
      // scrypt halves: keep the two in flight half a hash apart (the second waits until the first is half way), so
      // their phase-boundary polls interleave; re-established after every switch
      if (job->algo == Algo::kScrypt && scrypt_halves && fifo.size() == 1) {
        const Batch& only = slots[fifo.front()];
        if (only.epoch == epoch && monotonic_seconds() - only.enq_host < 0.5 * scrypt_hash_s) break;
      }
      int free_slot = -1;
      for (int i = 0; i < kInflight; ++i)
        if (!slots[i].busy) { free_slot = i; break; }
      if (free_slot < 0) break;
      enqueue(slots[free_slot], job, gen, fifo.empty() ? nullptr : &slots[fifo.back()]);
      fifo.push_back(free_slot);
      progressed = true;
    }
    if (!progressed) {
      if (!job && fifo.empty()) {
        uint64_t g2 = 0;
        (void)current_job(&g2);  // waits (<= 10 ms) for work instead of spinning
      } else {
        std::this_thread::sleep_for(kIdlePoll);
      }
    }
  }
  // drain: let the batches in flight finish (abort them first: the miner is stopping)
  if (!fifo.empty()) {
    ++epoch;
    try {
      write_abort(epoch);
    } catch (const std::exception&) {
      // a faulted device: the drain below reports it
    }
  }
  uint64_t gen = 0;
  auto job = peek_job(&gen, nullptr);
  while (!fifo.empty()) {
    Batch& b = slots[fifo.front()];
    OTD_HIP(hipEventSynchronize(b.done));
    finish(b, job, gen);
    fifo.pop_front();
  }
}

// ------------------------------------------------------------- direct launches
// Synchronous-free launch API for the Python ops layer (torch-owned buffers and
// streams): pointers and the stream arrive as integers. Hits go to the legacy
// device-memory slots after out[0]; no abort word.

static HitSink ops_sink(uintptr_t out, uint32_t cap, uint32_t words) {
  HitSink s;
  s.out = reinterpret_cast<uint32_t*>(out);
  s.cap = cap;
  s.words = words;
  return s;
}

void py_launch_sha256d(const Sha256dParams& p, uint32_t base, uint64_t count, uintptr_t out, uint32_t cap, int grid,
                       uintptr_t stream) {
  OTD_HIP(launch_sha256d_search(p, base, count, ops_sink(out, cap, 1), grid, reinterpret_cast<hipStream_t>(stream)));
}

void py_launch_sha256d_k(const Sha256dParamsK& p, uint32_t base, uint64_t count, uintptr_t out, uint32_t cap, int grid,
                         uintptr_t stream) {
  OTD_HIP(launch_sha256d_search_k(p, base, count, ops_sink(out, cap, 2), grid, reinterpret_cast<hipStream_t>(stream)));
}

void py_launch_sha256d_v(const Sha256dParamsV& p, uintptr_t vars, uint32_t base, uint64_t count, uintptr_t out,
                         uint32_t cap, int grid, uintptr_t stream, int block, int chains) {
  OTD_HIP(launch_sha256d_search_v(p, reinterpret_cast<const Sha256dVariant*>(vars), base, count,
                                  ops_sink(out, cap, 2), grid, reinterpret_cast<hipStream_t>(stream), block, chains));
}

void py_launch_scrypt(const ScryptParams& p, uint32_t base, uint32_t count, uintptr_t xbuf, uintptr_t scratch, int gap,
                      uintptr_t out, uint32_t cap, int grid, uintptr_t stream) {
  OTD_HIP(launch_scrypt_search(p, base, count, reinterpret_cast<void*>(xbuf), reinterpret_cast<void*>(scratch), gap,
                               ops_sink(out, cap, 1), grid, reinterpret_cast<hipStream_t>(stream)));
}

void py_launch_x11_stage(const X11Params& p, int stage, uint32_t base, uintptr_t H, uint32_t stride, uint32_t n,
                         uintptr_t out, uint32_t cap, uintptr_t stream) {
  const HitSink s = ops_sink(out, cap, 1);
  OTD_HIP(x11_launch_stage(stage, p, base, reinterpret_cast<uint64_t*>(H), stride, n, out ? &s : nullptr,
                           reinterpret_cast<hipStream_t>(stream)));
}

void py_launch_x11(const X11Params& p, uint32_t base, uintptr_t H, uint32_t stride, uint32_t n, uintptr_t out,
                   uint32_t cap, uintptr_t stream) {
  const HitSink s = ops_sink(out, cap, 1);
  OTD_HIP(x11_launch_chain(p, base, reinterpret_cast<uint64_t*>(H), stride, n, out ? &s : nullptr,
                           reinterpret_cast<hipStream_t>(stream)));
}

int gpu_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

std::string gpu_arch_name(int device) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return "";
  return prop.gcnArchName;
}

int gpu_cu_count(int device) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 0;
  return prop.multiProcessorCount;
}

}  // namespace otedama
