// Shared device/host helpers for the gfx950 kNN engine.
//
// Ordering keys: every candidate is a 64-bit composite
//     (order_key(distance) << 32) | global_row
// so that unsigned comparison of composites is the deterministic
// (distance asc, row asc) order of the C ABI contract (include/fenix_knn.h).
// Arrow's select_k_unstable (reference src/fenix/io/index/index.py:166-168)
// orders NaN after numbers; order_key maps every NaN to 0xFFFFFFFF and
// -0.0 to +0.0.  The all-ones composite is the "empty slot" sentinel.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fx {

constexpr int kWave = 64;
constexpr uint64_t kEmpty = ~0ull;

__host__ __device__ __forceinline__ uint32_t order_key(float f) {
#ifdef __HIP_DEVICE_COMPILE__
  uint32_t u = __float_as_uint(f);
#else
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
#endif
  if ((u & 0x7fffffffu) == 0u) u = 0u;                      // -0 -> +0
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0xffffffffu;  // NaN last
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__host__ __device__ __forceinline__ float key_float(uint32_t k) {
  uint32_t u = (k == 0xffffffffu) ? 0x7fc00000u : ((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
#ifdef __HIP_DEVICE_COMPILE__
  return __uint_as_float(u);
#else
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
#endif
}

__host__ __device__ __forceinline__ uint64_t make_comp(float dist, uint32_t row) {
  return ((uint64_t)order_key(dist) << 32) | (uint64_t)row;
}

// splitmix64 finaliser (Steele, Lea, Flood 2014) — the portable corpus generator.
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Irwin-Hall(4) of the four 16-bit fields, centred and scaled to unit variance.
// Integer sum is exact; one f32 multiply -> bit-identical on host and device.
__host__ __device__ __forceinline__ float irwin_hall4(uint64_t h) {
  int s = (int)(h & 0xffff) + (int)((h >> 16) & 0xffff) + (int)((h >> 32) & 0xffff) +
          (int)(h >> 48) - 131070;
  return (float)s * 2.6428998e-05f;  // sqrt(3) / 65536
}

}  // namespace fx
