// Native mining runtime: job templates with search-space rolling, the GPU and
// CPU miners (one host thread each driving launches / SHA-NI loops), and the
// bounded share queue the Python control plane polls.
//
// Parity:
//   * miner.Worker (internal/miner/worker.go:46-298): Start/Stop/SetWork/Stats,
//     non-blocking share send with a drop counter (worker.go:266-275), job
//     epochs (workVer, worker.go:94-96,231-237).
//   * Reference defects NOT reproduced: every device gets a
//     disjoint variant stripe instead of identical Work (engine/run.go:1294), and
//     the search space extends past 2^32 via extranonce2 / BIP320 version /
//     ntime rolling instead of silently wrapping (worker.go:279).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace otedama {

enum class Algo : int { kSha256d = 0, kScrypt = 1, kX11 = 2 };

// A pool job plus the rules for deriving header variants from it.
struct JobTemplate {
  uint64_t epoch = 0;       // bumped by the control plane on every new job / target
  std::string job_id;       // opaque pool job id (SV2: decimal u32, V1: hex string)
  uint32_t channel_id = 0;
  Algo algo = Algo::kSha256d;
  uint8_t header[80] = {0};  // version | prevhash | merkle | ntime | nbits | nonce(ignored)
  uint8_t target[32] = {0};  // share target, little-endian (byte 31 most significant)
  uint32_t version_mask = 0;  // BIP320 rollable version bits (0 = no version rolling)
  uint32_t ntime_roll = 0;    // max ntime offset (0 = no ntime rolling)
  // Stratum V1: coinbase = coinb1 | extranonce1 | extranonce2 | coinb2; merkle
  // root = fold(sha256d(coinbase), branches). Empty coinb1/coinb2 = fixed merkle.
  bool has_coinbase = false;
  std::vector<uint8_t> coinb1, coinb2, extranonce1;
  uint32_t extranonce2_size = 0;
  std::vector<std::vector<uint8_t>> merkle_branches;
  // Variant stripe owned by this device: v = variant_start + k * variant_stride.
  uint64_t variant_start = 0;
  uint64_t variant_stride = 1;

  uint64_t variant_space() const;
  // Materialises variant v: full 80-byte header (nonce 0) and the rolled fields.
  void variant_header(uint64_t v, uint8_t out[80], uint32_t* version, uint32_t* ntime,
                      uint64_t* extranonce2) const;
};

struct ShareRecord {
  uint64_t epoch;
  std::string job_id;
  uint32_t channel_id;
  uint32_t nonce;
  uint32_t ntime;
  uint32_t version;
  uint64_t extranonce2;
  uint32_t extranonce2_size;
  uint8_t hash[32];
  std::string device_id;
  double found_at = 0;         // CLOCK_MONOTONIC seconds when the host verified the share
  double device_found_at = 0;  // CLOCK_MONOTONIC seconds of the kernel's hit (s_memrealtime mapped to host time;
                               // 0 when the device did not stamp it, e.g. the CPU miner)
};

struct MinerStats {
  uint64_t hashes = 0;      // nonces searched (counted per launch, not per hash)
  uint64_t candidates = 0;  // kernel hits before host re-verification
  uint64_t shares = 0;      // verified shares queued
  uint64_t dropped = 0;     // shares dropped because the queue was full
  uint64_t launches = 0;
  uint64_t rejected_candidates = 0;  // top-word ties that failed the full compare
  uint64_t variant_launches = 0;     // SHA-256d launches that searched K > 1 header variants (shared block 2)
  double busy_seconds = 0;           // device (or thread) time spent hashing
  bool faulted = false;              // the device thread died on a HIP error
  std::string error;
  // Search-space cursor: first variant index of this device's stripe not yet started, and the control-plane epoch
  // of the job it belongs to (a re-split after a device / rank loss starts past every cursor of the current work
  // so nothing is searched twice).
  uint64_t variant_next = 0;
  uint64_t variant_epoch = 0;
  // Job switches (GPU): set_job() of new work -> the first batch of that work running on the device, in ms.
  uint64_t job_switches = 0;
  double last_job_switch_ms = 0;
  std::vector<double> job_switch_ms;  // most recent samples (<= 64)
  // (control-plane epoch, CLOCK_MONOTONIC seconds) at which the first batch of each new work started running on the
  // device (CPU: the first chunk claimed), most recent <= 64: a node correlates them with the pool's new-block time.
  std::vector<std::pair<uint64_t, double>> work_started;
  uint64_t aborted_launches = 0;      // batches stopped early by the device abort word
  uint64_t ring_hits = 0;             // hits consumed from the host-coherent ring while their launch was running
  // Candidates lost on the way to the share queue, each counted (the reference counts every dropped share,
  // internal/miner/worker.go:266-275): kernel hits past a launch's hit-ring capacity, and scrypt candidates refused
  // by the bounded host-verifier queue.
  uint64_t ring_overflow = 0;
  uint64_t verify_dropped = 0;
  uint64_t verify_queue_peak = 0;     // deepest the scrypt verifier queue has been
  uint64_t launch_hashes = 0;         // hashes per launch of the last batch (capped from the share target)
  double clock_calib_rtt_us = 0;      // round trip of the start-up device-clock calibration
  uint64_t clock_samples = 0;         // per-launch clock stamps folded into the device -> host clock mapping
  bool host_abort = false;            // the abort word is stored by the CPU through the BAR (no control stream)
  uint64_t reserved_cus = 0;          // CUs left out of the search streams' CU mask (OTEDAMA_RESERVE_CUS)
  // Device-timeline time (s, from the miner's start) at which the batches counted in `hashes` had completed: a
  // rate over two samples, (hashes1 - hashes0) / (done_at1 - done_at0), is exact instead of quantized by launches.
  double hashes_done_at_s = 0;
  // Start-up phases of the device thread, in order, each a duration in ms (GPU: hip_set_device, buffers,
  // clock_calibration, wait_first_job, first_batch = first job's set_job -> its first batch running).
  std::vector<std::pair<std::string, double>> startup_ms;
  std::vector<std::pair<std::string, double>> startup_rss_mb;  // process resident set after each phase (MiB)
};

// Full-target re-verification of a candidate (host SHA-256d / scrypt).
bool verify_share(Algo algo, const uint8_t header80[80], const uint8_t target[32], uint8_t hash_out[32]);
void scrypt_1024_1_1(const uint8_t header80[80], uint8_t out[32]);
// n scrypt(1024, 1, 1) hashes, eight at a time on AVX2 (one at a time without it).
void scrypt_1024_1_1_batch(int n, const uint8_t* const header80[], uint8_t* const out[]);
void merkle_root_from_coinbase(const JobTemplate& job, uint64_t extranonce2, uint8_t root_out[32]);

// Bounded share queue with an eventfd that becomes readable on every push, so a consumer (the asyncio engine
// through loop.add_reader, a device process's forwarder through poll) wakes on the share instead of polling.
class ShareQueue {
 public:
  explicit ShareQueue(size_t cap);
  ~ShareQueue();
  ShareQueue(const ShareQueue&) = delete;
  ShareQueue& operator=(const ShareQueue&) = delete;
  bool push(ShareRecord&& s);  // false (and counted) when full
  std::vector<ShareRecord> drain(size_t max);
  size_t size();
  uint64_t dropped() const { return dropped_.load(); }
  int event_fd() const { return efd_; }
 private:
  int efd_ = -1;
  std::mutex mu_;
  std::deque<ShareRecord> q_;
  size_t cap_;
  std::atomic<uint64_t> dropped_{0};
};

class MinerBase {
 public:
  MinerBase(std::string device_id, size_t queue_cap) : device_id_(std::move(device_id)), queue_(queue_cap) {}
  virtual ~MinerBase() = default;
  virtual void start() = 0;
  virtual void stop() = 0;
  // nullptr job = pause (curtailment / arbitration idles the device).
  void set_job(std::shared_ptr<const JobTemplate> job);
  std::vector<ShareRecord> poll(size_t max) { return queue_.drain(max); }
  MinerStats stats();
  const std::string& device_id() const { return device_id_; }
  int share_fd() const { return queue_.event_fd(); }

 protected:
  std::shared_ptr<const JobTemplate> current_job(uint64_t* gen);
  // Non-blocking: the current job, its work generation and when that generation was set (monotonic seconds).
  std::shared_ptr<const JobTemplate> peek_job(uint64_t* gen, double* set_at);
  std::string device_id_;
  ShareQueue queue_;
  std::mutex job_mu_;
  std::condition_variable job_cv_;
  std::shared_ptr<const JobTemplate> job_;
  std::shared_ptr<const JobTemplate> last_work_;  // last non-null job (work identity)
  uint64_t job_gen_ = 0;                          // bumps only when the search space changes
  double job_set_at_ = 0;                         // monotonic time of the last set_job that changed the work
  std::atomic<bool> running_{false};
  std::mutex stats_mu_;
  MinerStats stats_;
};

// One host thread per GPU: two batches in flight on a private HIP stream. Hits reach the host while a launch
// runs (host-coherent ring, otedama/hitsink.h); new work or a pause moves the device abort word so the
// obsolete batches stop within one grid-stride trip.
class GpuMiner : public MinerBase {
 public:
  // sha_variants: SHA-256d header variants per launch that share block 2 (version rolling): 128 (default) = the
  // two-chain version-parallel kernel (two variants per lane, sha256d_search_v2); 64 = one variant per lane of a
  // wave (sha256d_search_v); 1..16 = the K-variant kernel (rounded down to an instantiated K: 2, 3, 4, 6, 8, 12,
  // 16). A job whose variant space cannot supply that many variants with a common block 2 falls back to the next
  // smaller layout it can supply (128 -> 64 -> K).
  GpuMiner(int device, std::string device_id, uint64_t batch_nonces, int grid, size_t queue_cap,
           int sha_variants = 128);
  ~GpuMiner() override;
  void start() override;
  void stop() override;
 private:
  void loop();
  int device_;
  uint64_t batch_;
  int grid_;
  int sha_k_;
  bool sha_v_;   // version-parallel kernel enabled
  bool sha_v2_;  // two-chain version-parallel kernel enabled (tried first)
  int grid_k_ = 0;
  int grid_v_ = 0;
  int grid_v2_ = 0;
  double rt_offset_ = 0;  // host monotonic seconds at device realtime 0 (s_memrealtime, 100 MHz)
  std::thread th_;
};

// CPU SHA-256d miner: `threads` workers claiming 64Ki-nonce chunks (SHA-NI).
class CpuMiner : public MinerBase {
 public:
  CpuMiner(int threads, std::string device_id, size_t queue_cap);
  ~CpuMiner() override;
  void start() override;
  void stop() override;
 private:
  void loop(int tid);
  int threads_;
  std::vector<std::thread> ths_;
  std::atomic<uint64_t> cursor_{0};
  std::atomic<uint64_t> cursor_gen_{0};  // job_gen_ of the cursor; first job is gen 1
  std::mutex cursor_mu_;
};

// Single-thread CPU scan of [start, start+count) nonces (bench + tests).
// Returns the nonces (header byte order) whose SHA-256d meets the target.
std::vector<uint32_t> cpu_scan_sha256d(const uint8_t header80[80], const uint8_t target[32], uint32_t start,
                                       uint64_t count);
std::string cpu_scan_method();  // the CPU SHA-256d scan this host runs, e.g. "avx512 16 lanes x 2 groups"
std::vector<uint32_t> cpu_scan_sha256d_lanes(int lanes, const uint8_t header80[80], const uint8_t target[32],
                                             uint32_t start, uint64_t count);

// Seconds on CLOCK_MONOTONIC (same clock as Python time.monotonic()).
double monotonic_seconds();

// True when [lo, hi) lies inside one line of a /proc/<pid>/maps text whose permissions are read AND write. A range the
// GPU runtime reserved with PROT_NONE ("---p") does not qualify: the CPU would fault on its first store.
bool maps_range_writable(const std::string& maps, uintptr_t lo, uintptr_t hi);

}  // namespace otedama
