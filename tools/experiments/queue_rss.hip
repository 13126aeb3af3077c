// Which HIP call creates which hardware queue (one 173 MiB anonymous mapping each on gfx950, profiles/r4/c_host_abort)?
// Prints the resident set and the number of >= 160 MiB anonymous mappings after each step of a device process's
// start-up, in the order the GPU miner makes them. Run under GPU_MAX_HW_QUEUES=1 and without it.
// Build: hipcc --offload-arch=gfx950 -O2 tools/queue_rss.hip -o tools/bin/queue_rss
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <unistd.h>

static double rss_mb() {
  FILE* f = std::fopen("/proc/self/statm", "r");
  unsigned long size = 0, res = 0;
  if (!f || std::fscanf(f, "%lu %lu", &size, &res) != 2) return -1;
  std::fclose(f);
  return double(res) * double(sysconf(_SC_PAGESIZE)) / (1024.0 * 1024.0);
}

// anonymous mappings of at least 160 MiB (the hardware-queue areas)
static int big_anon() {
  FILE* f = std::fopen("/proc/self/maps", "r");
  if (!f) return -1;
  char line[512];
  int n = 0;
  while (std::fgets(line, sizeof line, f)) {
    unsigned long a = 0, b = 0;
    char path[256] = "";
    if (std::sscanf(line, "%lx-%lx %*s %*s %*s %*s %255s", &a, &b, path) >= 2 && path[0] == '\0' &&
        b - a >= (160ul << 20))
      ++n;
  }
  std::fclose(f);
  return n;
}

__global__ void touch(int* p) {
  if (threadIdx.x == 0) p[blockIdx.x] = 1;
}

static void step(const char* name) { std::printf(", \"%s\": [%.1f, %d]", name, rss_mb(), big_anon()); }

int main() {
  std::printf("{\"start\": [%.1f, %d]", rss_mb(), big_anon());
  if (hipSetDevice(0) != hipSuccess) return 1;
  step("set_device");
  if (hipFree(nullptr) != hipSuccess) return 1;
  step("context");
  int* d = nullptr;
  if (hipMalloc(&d, 1 << 20) != hipSuccess) return 1;
  step("malloc");
  int* h = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&h), 4096, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
    return 1;
  step("host_malloc");
  hipStream_t s0 = nullptr, s1 = nullptr;
  if (hipStreamCreateWithFlags(&s0, hipStreamNonBlocking) != hipSuccess) return 1;
  step("stream0");
  if (hipStreamCreateWithFlags(&s1, hipStreamNonBlocking) != hipSuccess) return 1;
  step("stream1");
  hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s0, d);
  if (hipStreamSynchronize(s0) != hipSuccess) return 1;
  step("launch_s0");
  hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s1, d);
  if (hipStreamSynchronize(s1) != hipSuccess) return 1;
  step("launch_s1");
  if (hipMemsetAsync(d, 0, 64, s0) != hipSuccess || hipStreamSynchronize(s0) != hipSuccess) return 1;
  step("memset_s0");
  if (hipMemcpyAsync(h, d, 64, hipMemcpyDeviceToHost, s0) != hipSuccess || hipStreamSynchronize(s0) != hipSuccess)
    return 1;
  step("memcpy_d2h_s0");
  if (hipMemset(d, 0, 64) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
  step("memset_null_stream");
  hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, nullptr, d);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  step("launch_null_stream");
  std::printf("}\n");
  (void)hipStreamDestroy(s0);
  (void)hipStreamDestroy(s1);
  (void)hipHostFree(h);
  (void)hipFree(d);
  return 0;
}
