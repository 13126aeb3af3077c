// GpuMiner: one host thread per GPU driving double-buffered search batches on a
// private HIP stream (short launches + pinned result buffers so a
// job switch or a found share is never more than ~one batch away).
//
// Per batch: hipMemsetAsync(hit counter) -> search kernel -> hipMemcpyAsync of
// the hit slots into pinned host memory -> event. While batch k runs on the GPU
// the thread re-verifies batch k-1's candidates on the CPU (full 256-bit compare)
// and queues shares tagged with the job epoch that produced them.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <string>

#include "otedama/job.h"
#include "otedama/runtime.h"
#include "otedama/sha256.h"
#include "otedama/trace.h"
#include "otedama/x11_launch.h"

namespace otedama {

hipError_t launch_sha256d_search(const Sha256dParams& p, uint32_t base, uint64_t count, uint32_t* out,
                                 uint32_t cap, int grid, hipStream_t stream);
hipError_t launch_sha256d_search_k(const Sha256dParamsK& p, uint32_t base, uint64_t count, uint32_t* out, uint32_t cap,
                                   int grid, hipStream_t stream);
hipError_t launch_sha256d_search_v(const Sha256dParamsV& p, const Sha256dVariant* vars, uint32_t base, uint64_t count,
                                   uint32_t* out, uint32_t cap, int grid, hipStream_t stream, int block = 256,
                                   int chains = 1);

hipError_t launch_scrypt_search(const ScryptParams& p, uint32_t base, uint32_t count, void* xbuf, void* scratch,
                                int gap, uint32_t* out, uint32_t cap, int grid, hipStream_t stream);
uint64_t scrypt_scratch_bytes(int grid, int gap);
int gpu_cu_count(int device);

#define OTD_HIP(call)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (call);                                                                        \
    if (e_ != hipSuccess)                                                                          \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " #call); \
  } while (0)

namespace {
constexpr uint32_t kHitCap = 1024;

struct Slot {
  uint32_t* d_out = nullptr;
  uint32_t* h_out = nullptr;
  hipEvent_t start{}, done{};
  bool busy = false;
  std::shared_ptr<const JobTemplate> job;
  uint64_t gen = 0;
  uint64_t count = 0;  // nonces per variant
  int nvar = 1;        // > 1: K-variant / version-parallel SHA-256d launch, hits carry the variant index
  uint8_t header[kSha256dV2Group][80];
  uint32_t version[kSha256dV2Group] = {0}, ntime[kSha256dV2Group] = {0};
  uint64_t en2[kSha256dV2Group] = {0};
  Sha256dVariant* d_vars = nullptr;  // version-parallel kernel: per-lane variant table (device)
  Sha256dVariant* h_vars = nullptr;  // pinned staging copy
  TraceId range = 0;  // roctx: enqueue -> host verification of this batch
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
  OTD_HIP(hipSetDevice(device_));
  hipStream_t stream = nullptr;
  Slot slots[2];
  // scrypt scratch (allocated lazily on the first scrypt job)
  void* scratch = nullptr;
  void* xbuf = nullptr;
  // X11 intermediate digests (8 u64 planes x batch), allocated on the first x11 job
  uint64_t* x11_h = nullptr;
  // Released on every exit, including a HIP error thrown mid-loop (device fault): in-flight
  // batches are drained first so nothing is freed under a running kernel or copy.
  struct Release {
    std::function<void()> f;
    ~Release() { f(); }
  } release{[&] {
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto& s : slots) {
      if (s.d_out) (void)hipFree(s.d_out);
      if (s.h_out) (void)hipHostFree(s.h_out);
      if (s.start) (void)hipEventDestroy(s.start);
      if (s.done) (void)hipEventDestroy(s.done);
      if (s.d_vars) (void)hipFree(s.d_vars);
      if (s.h_vars) (void)hipHostFree(s.h_vars);
    }
    if (scratch) (void)hipFree(scratch);
    if (xbuf) (void)hipFree(xbuf);
    if (x11_h) (void)hipFree(x11_h);
    if (stream) (void)hipStreamDestroy(stream);
  }};
  OTD_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  for (auto& s : slots) {
    OTD_HIP(hipMalloc(&s.d_out, (1 + 2 * kHitCap) * sizeof(uint32_t)));
    OTD_HIP(hipHostMalloc(&s.h_out, (1 + 2 * kHitCap) * sizeof(uint32_t), hipHostMallocDefault));
    OTD_HIP(hipEventCreate(&s.start));
    OTD_HIP(hipEventCreate(&s.done));
    if (sha_v_) {
      OTD_HIP(hipMalloc(&s.d_vars, kSha256dV2Group * sizeof(Sha256dVariant)));
      OTD_HIP(hipHostMalloc(&s.h_vars, kSha256dV2Group * sizeof(Sha256dVariant), hipHostMallocDefault));
    }
  }
  // Lane-cooperative full-line ROMix (gap 1, nt pad traffic, 16 blocks/CU = 128 GiB of HBM): ~16.75 MH/s vs
  // 13.6-14.0 for the per-lane kernels at gap 1/2 (profiles/r1/scrypt_romix_ab.md).
  const int scrypt_gap = kScryptCoop;
  const int scrypt_grid = (gpu_cu_count(device_) > 0 ? gpu_cu_count(device_) : 256) * 16;
  const uint32_t scrypt_batch = uint32_t(scrypt_grid) * 256u;
  // X11: eleven stage kernels per batch over a 64 B/nonce digest buffer (512 MiB at 2^23).
  const uint32_t x11_batch = 1u << 23;
  // K-variant SHA-256d kernel (K states per lane, 4-6 waves/SIMD): 16 blocks of 256 per CU
  // (tools/bench_sha_k.py sweeps K and the grid; profiles/r2/).
  grid_k_ = (gpu_cu_count(device_) > 0 ? gpu_cu_count(device_) : 256) * 16;
  // Version-parallel kernel (8-waves/SIMD build): 64 blocks of 256 per CU (tools/bench_sha_v.py, profiles/r2/sha_v).
  grid_v_ = (gpu_cu_count(device_) > 0 ? gpu_cu_count(device_) : 256) * 64;
  // Two-chain kernel (4 waves/SIMD build): 128 blocks of 256 per CU (tools/bench_sha_v.py --chains2-bpc,
  // profiles/r2/sha_v2).
  grid_v2_ = (gpu_cu_count(device_) > 0 ? gpu_cu_count(device_) : 256) * 128;
  // Host variant table of the current 64/128-variant group, rebuilt only when the group changes (once per 2^32
  // nonces).
  uint64_t v_table_gen = ~0ull, v_table_k = ~0ull;
  int v_table_n = 0;
  Sha256dParamsV v_params{};
  Sha256dVariant v_table[kSha256dV2Group];

  uint64_t cur_gen = ~0ull;
  uint64_t k = 0;       // variant-stripe position
  uint64_t nonce_off = 0;
  int which = 0;

  auto finish = [&](Slot& s) {
    if (!s.busy) return;
    OTD_HIP(hipEventSynchronize(s.done));
    trace_stop(s.range);
    float ms = 0;
    hipEventElapsedTime(&ms, s.start, s.done);
    const uint32_t n = s.h_out[0] < kHitCap ? s.h_out[0] : kHitCap;
    TraceScope verify_scope("otd.verify_candidates");
    uint64_t good = 0, bad = 0;
    const bool multi = s.nvar > 1;
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t nonce = multi ? s.h_out[1 + 2 * i] : s.h_out[1 + i];
      const uint32_t vi = multi ? s.h_out[2 + 2 * i] : 0u;
      if (vi >= (uint32_t)s.nvar) { ++bad; continue; }
      uint8_t hdr[80];
      std::memcpy(hdr, s.header[vi], 80);
      store_le32(hdr + 76, nonce);
      ShareRecord r{};
      if (!verify_share(s.job->algo, hdr, s.job->target, r.hash)) { ++bad; continue; }
      r.epoch = s.job->epoch; r.job_id = s.job->job_id; r.channel_id = s.job->channel_id;
      r.nonce = nonce; r.ntime = s.ntime[vi]; r.version = s.version[vi]; r.extranonce2 = s.en2[vi];
      r.extranonce2_size = s.job->extranonce2_size; r.device_id = device_id_;
      r.found_at = monotonic_seconds();
      queue_.push(std::move(r));
      ++good;
    }
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.hashes += s.count * (uint64_t)s.nvar;
    stats_.candidates += s.h_out[0];
    stats_.shares += good;
    stats_.rejected_candidates += bad;
    stats_.busy_seconds += ms * 1e-3;
    stats_.launches += 1;
    if (multi) stats_.variant_launches += 1;
    s.busy = false;
    s.job.reset();
  };

  while (running_.load()) {
    uint64_t gen = 0;
    auto job = current_job(&gen);
    if (!job) {
      finish(slots[which ^ 1]);
      continue;
    }
    if (gen != cur_gen) { cur_gen = gen; k = 0; nonce_off = 0; }
    const uint64_t v = job->variant_start + k * job->variant_stride;
    if (v >= job->variant_space()) {  // stripe exhausted; wait for fresh work
      finish(slots[which ^ 1]);
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
      continue;
    }
    Slot& s = slots[which];
    finish(s);  // slot reuse: make sure its previous batch is consumed
    s.job = job;
    s.gen = gen;
    s.nvar = 1;
    job->variant_header(v, s.header[0], &s.version[0], &s.ntime[0], &s.en2[0]);
    bool use_v = false;
    if (job->algo == Algo::kSha256d && sha_v_) {
      // 128 (two-chain kernel) or 64 consecutive stripe positions with a common block 2 -> one or two variants per
      // lane of the version-parallel kernel. A group is all-or-nothing (a shorter run takes the next layout down,
      // ending at the K path below) and depends only on (job, k), so every launch of a group uses the same kernel
      // and W3/nonce space.
      const int want = sha_v2_ ? kSha256dV2Group : kSha256dVGroup;
      int kv = 1;
      while (kv < want) {
        const uint64_t vk = job->variant_start + (k + kv) * job->variant_stride;
        if (vk >= job->variant_space()) break;
        job->variant_header(vk, s.header[kv], &s.version[kv], &s.ntime[kv], &s.en2[kv]);
        if (std::memcmp(s.header[kv] + 64, s.header[0] + 64, 12) != 0) break;
        ++kv;
      }
      if (kv >= kSha256dV2Group && sha_v2_) {
        use_v = true;
        s.nvar = kSha256dV2Group;
      } else if (kv >= kSha256dVGroup) {
        use_v = true;
        s.nvar = kSha256dVGroup;
      }
    }
    if (!use_v && job->algo == Algo::kSha256d && sha_k_ > 1) {
      // Group the next stripe positions whose headers differ only in block 1 (version rolling): they share
      // the block-2 message schedule in sha256d_search_k. Stops at the first one that differs in 64..75.
      int kv = 1;
      while (kv < sha_k_) {
        const uint64_t vk = job->variant_start + (k + kv) * job->variant_stride;
        if (vk >= job->variant_space()) break;
        job->variant_header(vk, s.header[kv], &s.version[kv], &s.ntime[kv], &s.en2[kv]);
        if (std::memcmp(s.header[kv] + 64, s.header[0] + 64, 12) != 0) break;
        ++kv;
      }
      s.nvar = sha256d_k_floor(kv);  // kernels exist for K in {2,3,4,6,8,12,16}
    }
    s.range = trace_start(job->algo == Algo::kScrypt ? "otd.scrypt.batch"
                          : job->algo == Algo::kX11  ? "otd.x11.batch"
                                                     : "otd.sha256d.batch");
    OTD_HIP(hipMemsetAsync(s.d_out, 0, sizeof(uint32_t), stream));
    OTD_HIP(hipEventRecord(s.start, stream));
    if (job->algo == Algo::kScrypt) {
      if (!scratch) {
        OTD_HIP(hipMalloc(&scratch, scrypt_scratch_bytes(scrypt_grid, scrypt_gap)));
        OTD_HIP(hipMalloc(&xbuf, uint64_t(scrypt_batch) * 128));
      }
      ScryptParams p;
      scrypt_prepare(s.header[0], job->target, &p);
      const uint64_t remaining = (1ull << 32) - nonce_off;
      s.count = remaining < scrypt_batch ? remaining : scrypt_batch;
      OTD_HIP(launch_scrypt_search(p, uint32_t(nonce_off), uint32_t(s.count), xbuf, scratch, scrypt_gap, s.d_out,
                                   kHitCap, scrypt_grid, stream));
    } else if (job->algo == Algo::kX11) {
      if (!x11_h) OTD_HIP(hipMalloc(&x11_h, uint64_t(x11_batch) * 64));
      X11Params p;
      x11_prepare(s.header[0], job->target, &p);
      const uint64_t remaining = (1ull << 32) - nonce_off;
      s.count = remaining < x11_batch ? remaining : x11_batch;
      OTD_HIP(x11_launch_chain(p, uint32_t(nonce_off), x11_h, x11_batch, uint32_t(s.count), s.d_out, kHitCap, stream));
    } else if (use_v) {
      const bool two = s.nvar == kSha256dV2Group;
      if (v_table_gen != gen || v_table_k != k || v_table_n != s.nvar) {
        const uint8_t* hs[kSha256dV2Group];
        for (int j = 0; j < s.nvar; ++j) hs[j] = s.header[j];
        if (!sha256d_prepare_v(hs, s.nvar, job->target, &v_params, v_table))
          throw std::runtime_error("sha256d_prepare_v");
        v_params.occupancy8 = two ? 0 : 1;  // two chains: the 4-waves/SIMD build; one chain: the 8-wave build
        v_table_gen = gen;
        v_table_k = k;
        v_table_n = s.nvar;
      }
      // The table is cached per (work, group) but a target-only update (SV2 SetTarget, V1 set_difficulty) keeps
      // the work generation: the share filter must follow the job's current target on every launch.
      v_params.target_hi = load_le32(job->target + 28);
      const size_t table_bytes = size_t(s.nvar) * sizeof(Sha256dVariant);
      std::memcpy(s.h_vars, v_table, table_bytes);
      OTD_HIP(hipMemcpyAsync(s.d_vars, s.h_vars, table_bytes, hipMemcpyHostToDevice, stream));
      // W3 (big-endian nonce word) windows tile [0, 2^32) exactly like the nonce windows of the other kernels;
      // the kernel reports nonce = bswap(W3). Launch duration stays batch_ hashes.
      s.count = batch_ >= uint64_t(s.nvar) ? batch_ / uint64_t(s.nvar) : 1;  // powers of two: still tiles 2^32
      OTD_HIP(launch_sha256d_search_v(v_params, s.d_vars, uint32_t(nonce_off), s.count, s.d_out, kHitCap,
                                      two ? grid_v2_ : grid_v_, stream, 256, two ? 2 : 1));
    } else if (s.nvar > 1) {
      Sha256dParamsK p;
      const uint8_t* hs[kSha256dMaxK];
      for (int j = 0; j < s.nvar; ++j) hs[j] = s.header[j];
      if (!sha256d_prepare_k(hs, s.nvar, job->target, &p)) throw std::runtime_error("sha256d_prepare_k");
      // Keep one launch's duration (job-switch latency) about independent of K: nonces per
      // variant = batch / (largest power of two <= K); batch is a power of two that tiles 2^32, so this
      // still tiles it.
      uint64_t div = 1;
      while (div * 2 <= (uint64_t)s.nvar && div * 2 <= batch_) div *= 2;
      s.count = batch_ / div;
      OTD_HIP(launch_sha256d_search_k(p, uint32_t(nonce_off), s.count, s.d_out, kHitCap, grid_k_, stream));
    } else {
      Sha256dParams p;
      sha256d_prepare(s.header[0], job->target, &p);
      s.count = batch_;
      OTD_HIP(launch_sha256d_search(p, uint32_t(nonce_off), s.count, s.d_out, kHitCap, grid_, stream));
    }
    OTD_HIP(hipMemcpyAsync(s.h_out, s.d_out, (1 + (s.nvar > 1 ? 2 : 1) * kHitCap) * sizeof(uint32_t),
                           hipMemcpyDeviceToHost, stream));
    OTD_HIP(hipEventRecord(s.done, stream));
    s.busy = true;
    nonce_off += s.count;
    if (nonce_off >= (1ull << 32)) { nonce_off = 0; k += (uint64_t)s.nvar; }
    which ^= 1;
    finish(slots[which]);  // consume the previous batch while this one runs
  }
  finish(slots[0]);
  finish(slots[1]);
}

// ------------------------------------------------------------- direct launches
// Synchronous-free launch API for the Python ops layer (torch-owned buffers and
// streams): pointers and the stream arrive as integers.

void py_launch_sha256d(const Sha256dParams& p, uint32_t base, uint64_t count, uintptr_t out, uint32_t cap, int grid,
                       uintptr_t stream) {
  OTD_HIP(launch_sha256d_search(p, base, count, reinterpret_cast<uint32_t*>(out), cap, grid,
                                reinterpret_cast<hipStream_t>(stream)));
}

void py_launch_sha256d_k(const Sha256dParamsK& p, uint32_t base, uint64_t count, uintptr_t out, uint32_t cap, int grid,
                         uintptr_t stream) {
  OTD_HIP(launch_sha256d_search_k(p, base, count, reinterpret_cast<uint32_t*>(out), cap, grid,
                                  reinterpret_cast<hipStream_t>(stream)));
}

void py_launch_sha256d_v(const Sha256dParamsV& p, uintptr_t vars, uint32_t base, uint64_t count, uintptr_t out,
                         uint32_t cap, int grid, uintptr_t stream, int block, int chains) {
  OTD_HIP(launch_sha256d_search_v(p, reinterpret_cast<const Sha256dVariant*>(vars), base, count,
                                  reinterpret_cast<uint32_t*>(out), cap, grid, reinterpret_cast<hipStream_t>(stream),
                                  block, chains));
}

void py_launch_scrypt(const ScryptParams& p, uint32_t base, uint32_t count, uintptr_t xbuf, uintptr_t scratch, int gap,
                      uintptr_t out, uint32_t cap, int grid, uintptr_t stream) {
  OTD_HIP(launch_scrypt_search(p, base, count, reinterpret_cast<void*>(xbuf), reinterpret_cast<void*>(scratch), gap,
                               reinterpret_cast<uint32_t*>(out), cap, grid, reinterpret_cast<hipStream_t>(stream)));
}

void py_launch_x11_stage(const X11Params& p, int stage, uint32_t base, uintptr_t H, uint32_t stride, uint32_t n,
                         uintptr_t out, uint32_t cap, uintptr_t stream) {
  OTD_HIP(x11_launch_stage(stage, p, base, reinterpret_cast<uint64_t*>(H), stride, n, reinterpret_cast<uint32_t*>(out),
                           cap, reinterpret_cast<hipStream_t>(stream)));
}

void py_launch_x11(const X11Params& p, uint32_t base, uintptr_t H, uint32_t stride, uint32_t n, uintptr_t out,
                   uint32_t cap, uintptr_t stream) {
  OTD_HIP(x11_launch_chain(p, base, reinterpret_cast<uint64_t*>(H), stride, n, reinterpret_cast<uint32_t*>(out), cap,
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
