// fetch_calib.hip — calibration of the gfx950 memory-side traffic counters (FETCH_SIZE /
// WRITE_SIZE and the TCC_EA0_* request counters rocprofv3 derives them from) against KNOWN byte
// counts in the access patterns the pafreport / GapAssem kernels use.
//
// Every kernel touches a 2 GiB buffer (8x the 256 MiB Infinity Cache) in one pattern, each cache
// line at most once per launch, and is launched once per process; profiles/calib/calibrate.py
// divides the counters of each launch by the pattern's known bytes.
//   stream16      coalesced streaming read, 16 B per lane (the guide's "1/2" case)
//   scatter4_128  4 B per lane, one lane per 128-B line, lines in a permuted order
//   scatter16_128 16 B per lane, one lane per 128-B line, permuted
//   scatter4_64   4 B per lane, one lane per 64-B half line (both halves of every line, far apart)
//   gather16      16 B per lane, every 16-B piece of the buffer once, in a permuted order
//   win48         48 B per lane (three 16-B loads), windows at 16-B offsets of permuted 256-B blocks,
//                 one per 128-B line (render's per-lane query windows)
//   store16       coalesced streaming store, 16 B per lane
//   store16_nt    the same with the non-temporal cache policy (render's report text)
//   scatter_st16  16 B store per lane, one per 128-B line, permuted
// Build: hipcc -O3 --offload-arch=gfx950 fetch_calib.hip -o fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t perm(uint64_t i, uint64_t n) {  // bijection on [0, n), n a power of 2
  return (i * 0x9E3779B97F4A7C15ull) & (n - 1);
}

__global__ void stream16(const v4u* __restrict__ a, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const v4u v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
template <int BYTES, int LINE>
__global__ void scatter(const uint8_t* __restrict__ a, uint64_t n_lines, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_lines; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t* p = a + perm(i, n_lines) * LINE;
    if (BYTES == 4) {
      acc ^= *reinterpret_cast<const uint32_t*>(p);
    } else {
      const v4u v = *reinterpret_cast<const v4u*>(p);
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void win48(const uint8_t* __restrict__ a, uint64_t n_lines, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_lines; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t l = perm(i, n_lines);
    // a 48-byte window at a 16-B-aligned offset 16 * (i % 8) of a 256-B block: offsets 96 and 112
    // cross into the block's second 128-B line
    const v4u* p = reinterpret_cast<const v4u*>(a + l * 256 + 16 * (i % 8));
    const v4u v0 = p[0], v1 = p[1], v2 = p[2];
    acc ^= v0.x ^ v1.y ^ v2.z ^ v0.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
template <int NT>
__global__ void store16(v4u* a, uint64_t n16) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const v4u v = {(uint32_t)i, 1u, 2u, 3u};
    if (NT) __builtin_nontemporal_store(v, a + i);
    else a[i] = v;
  }
}
__global__ void scatter_st16(uint8_t* a, uint64_t n_lines) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_lines; i += (uint64_t)gridDim.x * blockDim.x) {
    const v4u v = {(uint32_t)i, 1u, 2u, 3u};
    *reinterpret_cast<v4u*>(a + perm(i, n_lines) * 128) = v;
  }
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main() {
  const uint64_t N = 2ull << 30;  // bytes
  uint8_t* a = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&a, N));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 1, N));
  CK(hipDeviceSynchronize());
  const dim3 g(256 * 64), b(256);
  const uint64_t L128 = N / 128, L64 = N / 64;
  // name, requested bytes, distinct 128-B lines' bytes
  printf("{\"buffer_bytes\": %llu, \"kernels\": {\n", (unsigned long long)N);
  hipLaunchKernelGGL(stream16, g, b, 0, 0, (const v4u*)a, N / 16, out);
  printf(" \"stream16\": {\"requested\": %llu, \"lines128\": %llu},\n", (unsigned long long)N, (unsigned long long)N);
  hipLaunchKernelGGL((scatter<4, 128>), g, b, 0, 0, a, L128, out);
  printf(" \"scatter4_128\": {\"requested\": %llu, \"lines128\": %llu},\n", (unsigned long long)(4 * L128), (unsigned long long)N);
  hipLaunchKernelGGL((scatter<16, 128>), g, b, 0, 0, a, L128, out);
  printf(" \"scatter16_128\": {\"requested\": %llu, \"lines128\": %llu},\n", (unsigned long long)(16 * L128), (unsigned long long)N);
  hipLaunchKernelGGL((scatter<4, 64>), g, b, 0, 0, a, L64, out);
  printf(" \"scatter4_64\": {\"requested\": %llu, \"lines128\": %llu},\n", (unsigned long long)(4 * L64), (unsigned long long)N);
  hipLaunchKernelGGL((scatter<16, 16>), g, b, 0, 0, a, N / 16, out);
  printf(" \"gather16\": {\"requested\": %llu, \"lines128\": %llu},\n", (unsigned long long)N, (unsigned long long)N);
  hipLaunchKernelGGL(win48, g, b, 0, 0, a, N / 256, out);
  // (per 8 windows: 6 touch one 128-B line, 2 touch two)
  printf(" \"win48\": {\"requested\": %llu, \"lines128\": %llu},\n", (unsigned long long)(48 * (N / 256)),
         (unsigned long long)((N / 256) / 8 * 10 * 128));
  hipLaunchKernelGGL((store16<0>), g, b, 0, 0, (v4u*)a, N / 16);
  printf(" \"store16\": {\"requested\": %llu, \"lines128\": %llu},\n", (unsigned long long)N, (unsigned long long)N);
  hipLaunchKernelGGL((store16<1>), g, b, 0, 0, (v4u*)a, N / 16);
  printf(" \"store16_nt\": {\"requested\": %llu, \"lines128\": %llu},\n", (unsigned long long)N, (unsigned long long)N);
  hipLaunchKernelGGL(scatter_st16, g, b, 0, 0, a, L128);
  printf(" \"scatter_st16\": {\"requested\": %llu, \"lines128\": %llu}\n", (unsigned long long)(16 * L128), (unsigned long long)N);
  printf("}}\n");
  CK(hipDeviceSynchronize());
  CK(hipFree(a));
  CK(hipFree(out));
  return 0;
}
