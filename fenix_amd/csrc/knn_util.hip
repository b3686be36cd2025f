// Synthetic corpus generator and (dist,row) -> composite encoder.
//
// The generator is the device half of the portable generator whose host half
// is oracle/knn_ref.c (fx_ref_fill) and oracle/oracle.py (fill_normal); the
// two are bit-identical by construction (integer hash + one f32 multiply,
// an opaque barrier in the clustered variant so nothing is contracted
// into an FMA).  The clustered variant is the distribution of the reference's
// own test corpus, tests/test_flight.py:21-22 (x = x + 10 * x[0, :] per batch).
#include "fx_internal.h"

namespace fx {

template <typename T>
__global__ void __launch_bounds__(256)
    fill_kernel(T* __restrict__ x, int64_t n, int64_t d, uint64_t seed, int64_t row_base,
                int64_t cluster) {
  const uint64_t smix = seed * 0x9E3779B97F4A7C15ull;
  for (int64_t r = blockIdx.x; r < n; r += gridDim.x) {
    const uint64_t g = (uint64_t)(row_base + r);
    const uint64_t b0 = cluster > 0 ? g / (uint64_t)cluster * (uint64_t)cluster : g;
    for (int64_t c = threadIdx.x; c < d; c += blockDim.x) {
      float v = irwin_hall4(splitmix64(smix + g * (uint64_t)d + (uint64_t)c));
      if (cluster > 0) {
        const float v0 = irwin_hall4(splitmix64(smix + b0 * (uint64_t)d + (uint64_t)c));
        float t = 10.0f * v0;
        asm volatile("" : "+v"(t));  // opaque: keeps the product rounded before the add
        v = v + t;
      }
      x[r * d + c] = (T)v;
    }
  }
}

__global__ void __launch_bounds__(256)
    encode_kernel(const float* __restrict__ dist, const int64_t* __restrict__ row, int64_t count,
                  uint64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < count;
       i += (int64_t)gridDim.x * 256) {
    const int64_t r = row[i];
    out[i] = (r < 0 || r >= 0xffffffffll) ? kEmpty : make_comp(dist[i], (uint32_t)r);
  }
}

int launch_fill(void* x, int dtype, int64_t n, int64_t d, uint64_t seed, int64_t row_base,
                int64_t cluster, hipStream_t stream) {
  int64_t blocks = n < 65536 ? n : 65536;
  if (blocks < 1) return FX_OK;
  if (dtype == FX_DTYPE_F32) {
    hipLaunchKernelGGL(fill_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, stream,
                       reinterpret_cast<float*>(x), n, d, seed, row_base, cluster);
  } else {
    hipLaunchKernelGGL(fill_kernel<_Float16>, dim3((unsigned)blocks), dim3(256), 0, stream,
                       reinterpret_cast<_Float16*>(x), n, d, seed, row_base, cluster);
  }
  return check_launch("fill_kernel");
}

int launch_encode(const float* dist, const int64_t* row, int64_t count, uint64_t* out,
                  hipStream_t stream) {
  int64_t blocks = (count + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) return FX_OK;
  hipLaunchKernelGGL(encode_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, dist, row, count,
                     out);
  return check_launch("encode_kernel");
}

}  // namespace fx
