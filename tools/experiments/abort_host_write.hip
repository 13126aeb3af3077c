// Can the host move the miner's abort word without a HIP stream (and the ~190 MB hardware queue behind it)?
//
// The production miner writes its uncached device abort word with hipStreamWriteValue32 on a high-priority control
// stream (csrc/runtime/gpu_miner.hip). That stream is one of the three hardware queues a device process holds, and
// every queue costs ~190 MB of host memory (profiles/r3/o_rss). If the CPU can store to the word directly (VRAM
// mapped through the PCIe BAR: hsa_amd_agents_allow_access for the CPU agent), no control queue is needed for it.
//
// Per candidate allocation (hipDeviceMallocUncached, hipDeviceMallocFinegrained, and the GPU's fine-grained HSA pool)
// this prints the pool's CPU access rule, whether allow_access for the CPU succeeds, whether the range then shows up in
// /proc/self/maps (checked before the CPU touches it), and, when it does, the latency from a CPU store to a polling
// wave seeing it (the poll loop is bounded: every launch ends by itself within ~1 s). For comparison the same
// latency through hipStreamWriteValue32 on a high-priority stream. RSS (MiB) after each step.
//
// Build: hipcc --offload-arch=gfx950 -O2 tools/abort_host_write.hip -o tools/bin/abort_host_write -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

static double rss_mb() {
  FILE* f = std::fopen("/proc/self/statm", "r");
  unsigned long size = 0, res = 0;
  if (!f || std::fscanf(f, "%lu %lu", &size, &res) != 2) return -1;
  std::fclose(f);
  return double(res) * double(sysconf(_SC_PAGESIZE)) / (1024.0 * 1024.0);
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Is [p, p+n) inside a mapping of this process's CPU address space?
static bool cpu_mapped(const void* p, size_t n) {
  FILE* f = std::fopen("/proc/self/maps", "r");
  if (!f) return false;
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p), hi = lo + n;
  char line[512];
  bool ok = false;
  while (std::fgets(line, sizeof line, f)) {
    unsigned long a = 0, b = 0;
    if (std::sscanf(line, "%lx-%lx", &a, &b) == 2 && a <= lo && hi <= b) {
      ok = true;
      break;
    }
  }
  std::fclose(f);
  return ok;
}

// One lane polls the word until it equals `want` or max_iter polls have passed (bounded: the launch always ends).
__global__ void poll_word(const uint32_t* w, uint32_t want, uint64_t* out, uint32_t max_iter) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t i = 0;
  for (; i < max_iter; ++i) {
    if (__hip_atomic_load(const_cast<uint32_t*>(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == want) break;
    __builtin_amdgcn_s_sleep(4);
  }
  out[0] = t0;
  out[1] = __builtin_amdgcn_s_memrealtime();
  out[2] = i;
  out[3] = 1;
}

struct Ctx {
  hsa_agent_t cpu{}, gpu{};
  bool have_cpu = false, have_gpu = false;
  hsa_amd_memory_pool_t fine{};
  bool have_fine = false;
};

static hsa_status_t pick_pool(hsa_amd_memory_pool_t pool, void* data) {
  auto* c = static_cast<Ctx*>(data);
  hsa_amd_segment_t seg;
  uint32_t flags = 0;
  if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  hsa_amd_memory_pool_access_t acc = HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED;
  if (c->have_cpu) hsa_amd_agent_memory_pool_get_info(c->cpu, pool, HSA_AMD_AGENT_MEMORY_POOL_INFO_ACCESS, &acc);
  size_t sz = 0;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SIZE, &sz);
  std::printf("{\"gpu_pool_flags\": %u, \"size_gib\": %.1f, \"cpu_access\": %d}\n", flags, sz / 1073741824.0, int(acc));
  if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !c->have_fine) {
    c->fine = pool;
    c->have_fine = true;
  }
  return HSA_STATUS_SUCCESS;
}

static hsa_status_t pick_agent(hsa_agent_t a, void* data) {
  auto* c = static_cast<Ctx*>(data);
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_CPU && !c->have_cpu) { c->cpu = a; c->have_cpu = true; }
  if (t == HSA_DEVICE_TYPE_GPU && !c->have_gpu) { c->gpu = a; c->have_gpu = true; }
  return HSA_STATUS_SUCCESS;
}

// Launch the poller on `s`, move the word after 20 ms (host store, or hipStreamWriteValue32 on `ctl`), report the
// device-side time from the store to the poller seeing it.
static void measure(const char* name, uint32_t* word, bool host_store, hipStream_t s, hipStream_t ctl, uint64_t* out,
                    uint64_t* out_dev) {
  std::vector<double> lat_us;
  for (int rep = 0; rep < 8; ++rep) {
    const uint32_t want = 100 + rep;
    std::memset(out, 0, 4 * sizeof(uint64_t));
    const double t_launch = now_s();
    hipLaunchKernelGGL(poll_word, dim3(1), dim3(64), 0, s, word, want, out_dev, 1u << 20);
    if (hipGetLastError() != hipSuccess) { std::printf("{\"%s\": \"launch failed\"}\n", name); return; }
    // wait until the poller is running (out[0] is written at the end only, so just give it time to start)
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    const double t_store = now_s();
    if (host_store) {
      __atomic_store_n(word, want, __ATOMIC_RELEASE);
      __builtin_ia32_sfence();
    } else {
      (void)hipStreamWriteValue32(ctl, word, want, 0);
    }
    if (hipStreamSynchronize(s) != hipSuccess) { std::printf("{\"%s\": \"sync failed\"}\n", name); return; }
    const double t_done = now_s();
    const volatile uint64_t* o = out;
    const double dev_run_us = double(o[1] - o[0]) / 100.0;  // 100 MHz realtime
    // the poller starts a few us after the launch call, so store -> seen <= device run - (store - launch)
    const double seen_us = dev_run_us - (t_store - t_launch) * 1e6;
    lat_us.push_back(seen_us);
    std::printf("{\"%s\": {\"rep\": %d, \"polls\": %llu, \"device_run_us\": %.1f, \"store_to_seen_us_max\": %.1f, "
                "\"host_store_to_sync_us\": %.1f}}\n",
                name, rep, (unsigned long long)o[2], dev_run_us, seen_us, (t_done - t_store) * 1e6);
  }
}

int main() {
  std::printf("{\"start_mib\": %.1f}\n", rss_mb());
  if (hipSetDevice(0) != hipSuccess || hipFree(nullptr) != hipSuccess) return 1;
  std::printf("{\"context_mib\": %.1f}\n", rss_mb());
  Ctx c;
  hsa_iterate_agents(pick_agent, &c);
  if (!c.have_cpu || !c.have_gpu) { std::printf("{\"error\": \"no cpu/gpu agent\"}\n"); return 1; }
  hsa_amd_agent_iterate_memory_pools(c.gpu, pick_pool, &c);

  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  std::printf("{\"one_stream_mib\": %.1f}\n", rss_mb());
  uint64_t* out = nullptr;
  uint64_t* out_dev = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&out), 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return 1;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&out_dev), out, 0) != hipSuccess) return 1;

  struct Cand { const char* name; uint32_t* p; };
  std::vector<Cand> cands;
  uint32_t* p_unc = nullptr;
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&p_unc), 4096, hipDeviceMallocUncached) == hipSuccess)
    cands.push_back({"hip_uncached", p_unc});
  uint32_t* p_fg = nullptr;
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&p_fg), 4096, hipDeviceMallocFinegrained) == hipSuccess)
    cands.push_back({"hip_finegrained", p_fg});
  uint32_t* p_pool = nullptr;
  if (c.have_fine && hsa_amd_memory_pool_allocate(c.fine, 4096, 0, reinterpret_cast<void**>(&p_pool)) == HSA_STATUS_SUCCESS) {
    hsa_amd_agents_allow_access(1, &c.gpu, nullptr, p_pool);
    cands.push_back({"hsa_fine_pool", p_pool});
  }
  for (auto& k : cands) {
    (void)hipMemset(k.p, 0, 4096);
    (void)hipDeviceSynchronize();
    hipPointerAttribute_t attr{};
    const hipError_t ae = hipPointerGetAttributes(&attr, k.p);
    hsa_amd_pointer_info_t info{};
    info.size = sizeof(info);
    const hsa_status_t ie = hsa_amd_pointer_info(k.p, &info, nullptr, nullptr, nullptr);
    const bool mapped_before = cpu_mapped(k.p, 4);
    const hsa_status_t allow = hsa_amd_agents_allow_access(1, &c.cpu, nullptr, k.p);
    const bool mapped_after = cpu_mapped(k.p, 4);
    std::printf("{\"%s\": {\"hip_attr_rc\": %d, \"hip_type\": %d, \"hip_host_ptr\": \"%p\", \"hsa_info_rc\": %d, "
                "\"hsa_type\": %d, \"hsa_host_base\": \"%p\", \"cpu_mapped_before\": %s, \"allow_cpu_rc\": %d, "
                "\"cpu_mapped_after\": %s, \"rss_mib\": %.1f}}\n",
                k.name, int(ae), int(attr.type), attr.hostPointer, int(ie), int(info.type), info.hostBaseAddress,
                mapped_before ? "true" : "false", int(allow), mapped_after ? "true" : "false", rss_mb());
    if (mapped_after) measure(k.name, k.p, true, s, nullptr, out, out_dev);
  }
  // Baseline: the production form (hipStreamWriteValue32 on a high-priority stream) on the uncached word.
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  hipStream_t ctl = nullptr;
  if (p_unc && hipStreamCreateWithPriority(&ctl, hipStreamNonBlocking, hi) == hipSuccess) {
    std::printf("{\"with_control_stream_mib\": %.1f}\n", rss_mb());
    (void)hipMemset(p_unc, 0, 4096);
    (void)hipDeviceSynchronize();
    measure("stream_write_value", p_unc, false, s, ctl, out, out_dev);
  }
  (void)hipDeviceSynchronize();
  std::printf("{\"end_mib\": %.1f}\n", rss_mb());
  return 0;
}
