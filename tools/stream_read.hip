// Measured stream-read ceiling for the roofline: reads a buffer once with
// 16-byte loads (optionally nontemporal), XOR-folds so nothing is dead code,
// one dword per block out.  Not part of the product.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ void __launch_bounds__(256) stream_read(const u32x4* __restrict__ p, int64_t n16,
                                                   uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * 256 * 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 * 4 + threadIdx.x; i < n16; i += stride) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = i + u * 256;
      if (j < n16) {
        if constexpr (NT) v[u] = __builtin_nontemporal_load(p + j);
        else v[u] = p[j];
      } else {
        v[u] = u32x4(0);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

extern "C" int stream_read_launch(const void* p, int64_t bytes, void* out, int blocks, int nt,
                                  void* stream) {
  const int64_t n16 = bytes / 16;
  if (nt)
    hipLaunchKernelGGL(stream_read<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4*)p, n16, (uint32_t*)out);
  else
    hipLaunchKernelGGL(stream_read<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4*)p, n16, (uint32_t*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
