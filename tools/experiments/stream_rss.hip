// Resident set per HIP stream on gfx950 (the ~1 GB of host memory a device process gains when the miner creates
// its streams, profiles/r3/n_rss). Creates streams one at a time and prints the RSS after each, then launches one
// tiny kernel per stream (hardware queues are created lazily on first use in some runtimes).
// Build: hipcc --offload-arch=gfx950 -O2 tools/stream_rss.hip -o tools/bin/stream_rss
#include <hip/hip_runtime.h>

#include <cstdio>
#include <unistd.h>

static double rss_mb() {
  FILE* f = std::fopen("/proc/self/statm", "r");
  unsigned long size = 0, res = 0;
  if (!f || std::fscanf(f, "%lu %lu", &size, &res) != 2) return -1;
  std::fclose(f);
  return double(res) * double(sysconf(_SC_PAGESIZE)) / (1024.0 * 1024.0);
}

__global__ void touch(int* p) {
  if (threadIdx.x == 0) p[blockIdx.x] = 1;
}

int main() {
  std::printf("{\"start\": %.1f", rss_mb());
  if (hipSetDevice(0) != hipSuccess || hipFree(nullptr) != hipSuccess) return 1;
  std::printf(", \"context\": %.1f", rss_mb());
  int* d = nullptr;
  if (hipMalloc(&d, 64 * sizeof(int)) != hipSuccess) return 1;
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  hipStream_t s[6];
  for (int i = 0; i < 6; ++i) {
    const int prio = i < 4 ? lo : hi;
    if (hipStreamCreateWithPriority(&s[i], hipStreamNonBlocking, prio) != hipSuccess) return 1;
    std::printf(", \"stream%d_%s\": %.1f", i, i < 4 ? "normal" : "high", rss_mb());
    hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s[i], d);
    if (hipStreamSynchronize(s[i]) != hipSuccess) return 1;
    std::printf(", \"stream%d_used\": %.1f", i, rss_mb());
  }
  std::printf("}\n");
  for (auto& x : s) (void)hipStreamDestroy(x);
  (void)hipFree(d);
  return 0;
}
