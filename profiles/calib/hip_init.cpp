// hip_init.cpp — where the HIP runtime's start-up goes on the GPU box (the CLI's critical path,
// DESIGN.md §6 round 6): wall time of each first call, in order.
// Build: hipcc -O2 hip_init.cpp -o hip_init
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
  const double t0 = now();
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  const double t1 = now();
  e = hipSetDevice(0);
  const double t2 = now();
  e = hipFree(nullptr);
  const double t3 = now();
  hipStream_t st;
  e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  const double t4 = now();
  void* d = nullptr;
  e = hipMalloc(&d, 64 << 20);
  const double t5 = now();
  void* h = nullptr;
  e = hipHostMalloc(&h, 32 << 20, hipHostMallocDefault);
  const double t6 = now();
  e = hipMemcpyAsync(d, h, 1 << 20, hipMemcpyHostToDevice, st);
  e = hipStreamSynchronize(st);
  const double t7 = now();
  printf("devices %d: getDeviceCount %.1f ms, setDevice %.1f, free(0) %.1f, streamCreate %.1f, malloc 64MB %.1f, "
         "hostMalloc 32MB %.1f, first copy %.1f, total %.1f ms (%s)\n",
         n, 1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2), 1e3 * (t4 - t3), 1e3 * (t5 - t4), 1e3 * (t6 - t5),
         1e3 * (t7 - t6), 1e3 * (t7 - t0), hipGetErrorString(e));
  return 0;
}
