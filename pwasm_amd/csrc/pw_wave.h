// pw_wave.h — wave64 primitives on DPP (gfx950): inclusive prefix sums without LDS round trips.
// __shfl_up lowers to ds_bpermute (an LDS-latency round trip per step); these lower to
// v_add_u32_dpp row_shr:1/2/4/8 within each 16-lane row, then row_bcast:15 / row_bcast:31 to
// carry across rows (GFX9 DPP controls, present on CDNA4).
#ifndef PW_WAVE_H
#define PW_WAVE_H
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>

namespace pw {

template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint32_t dpp_or_zero(uint32_t v) {
  // lanes whose DPP source is outside the row (or masked) read 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xF, false);
}

// inclusive prefix sum over the 64 lanes (every lane active)
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t v) {
  v += dpp_or_zero<0x111>(v);        // row_shr:1
  v += dpp_or_zero<0x112>(v);        // row_shr:2
  v += dpp_or_zero<0x114>(v);        // row_shr:4
  v += dpp_or_zero<0x118>(v);        // row_shr:8
  v += dpp_or_zero<0x142, 0xA>(v);   // row_bcast:15 -> rows 1, 3
  v += dpp_or_zero<0x143, 0xC>(v);   // row_bcast:31 -> rows 2, 3
  return v;
}
__device__ __forceinline__ int wave_scan_incl(int v) { return (int)wave_scan_incl((uint32_t)v); }

// inclusive prefix minimum over the 64 lanes (every lane active); lanes whose DPP source is
// outside the row keep INT_MAX (the identity)
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ int dpp_or_max(int v) {
  return __builtin_amdgcn_update_dpp(INT_MAX, v, CTRL, ROW_MASK, 0xF, false);
}
__device__ __forceinline__ int wave_min_incl(int v) {
  v = min(v, dpp_or_max<0x111>(v));
  v = min(v, dpp_or_max<0x112>(v));
  v = min(v, dpp_or_max<0x114>(v));
  v = min(v, dpp_or_max<0x118>(v));
  v = min(v, dpp_or_max<0x142, 0xA>(v));
  v = min(v, dpp_or_max<0x143, 0xC>(v));
  return v;
}

// value of lane 63 (wave-uniform)
__device__ __forceinline__ uint32_t wave_last(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 63); }
__device__ __forceinline__ int wave_last(int v) { return __builtin_amdgcn_readlane(v, 63); }

}  // namespace pw
#endif
