// Wavefront (64-lane) primitives shared by the scan and merge kernels.
#pragma once

#include "fx_common.h"

namespace fx {

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum over each aligned group of 16 lanes; every lane of the group gets the
// same bits (each step adds a symmetric pair).
__device__ __forceinline__ float sum16(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return v;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    uint32_t t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  uint32_t lo = __shfl_xor((uint32_t)v, m);
  uint32_t hi = __shfl_xor((uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    uint64_t o = shfl_xor_u64(v, m);
    v = o > v ? o : v;
  }
  return v;
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

// Histogram add that collapses to one LDS atomic when every active lane of
// the wave targets the same bin (the common case for the leading key bytes,
// where all candidates share an exponent).  Must be called wave-uniformly.
__device__ __forceinline__ void hist_add(uint32_t* hist, uint32_t bin, bool active) {
  const uint64_t act = __ballot(active);
  if (act == 0) return;
  const int first = __ffsll((unsigned long long)act) - 1;
  const uint32_t b0 = __shfl(bin, first);
  const uint64_t same = __ballot(active && bin == b0);
  if (same == act) {
    if ((int)(threadIdx.x & 63) == first) atomicAdd(&hist[b0], (uint32_t)__popcll(act));
  } else if (active) {
    atomicAdd(&hist[bin], 1u);
  }
}

}  // namespace fx
