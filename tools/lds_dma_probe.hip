// Probe: does buffer_load ... lds (LDS-DMA) reach LDS offsets at and above
// 64 KB on gfx950?  Each of 8 waves DMAs 1 KB of known bytes to LDS offset
// base + wave KB, the workgroup reads them back with ds_read and counts
// mismatches.  hipcc --offload-arch=gfx950 -O2 tools/lds_dma_probe.hip -o tools/lds_dma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(3))) void* lds_ptr;

__global__ void __launch_bounds__(512) probe(const uint32_t* src, int base, uint32_t* bad) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < 160 * 1024 / 4; i += 512) reinterpret_cast<uint32_t*>(smem)[i] = 0xdeadbeefu;
  __syncthreads();
  const uint64_t p = reinterpret_cast<uint64_t>(src);
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(p), 0, 8 * 1024, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr)(smem + base + wid * 1024), 16,
                                           (uint32_t)lane * 16u, wid * 1024, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  uint32_t n = 0;
  for (int i = tid; i < 8 * 256; i += 512) {
    const uint32_t v = reinterpret_cast<const uint32_t*>(smem + base)[i];
    if (v != src[i]) ++n;
  }
  atomicAdd(bad, n);
}

int main() {
  uint32_t* src;
  uint32_t* bad;
  hipMalloc(&src, 8 * 1024);
  hipMalloc(&bad, 4);
  uint32_t h[2048];
  for (int i = 0; i < 2048; ++i) h[i] = 0x12340000u + i * 7u;
  hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice);
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  const int bases[] = {0, 32768, 57344, 61440, 63488, 65536, 69632, 98304, 131072, 151552};
  for (int b : bases) {
    hipMemset(bad, 0, 4);
    probe<<<1, 512, 160 * 1024>>>(src, b, bad);
    hipError_t e = hipDeviceSynchronize();
    uint32_t nb = 0;
    hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost);
    printf("{\"base\": %d, \"end\": %d, \"mismatches\": %u, \"err\": \"%s\"}\n", b, b + 8192, nb,
           hipGetErrorString(e));
  }
  return 0;
}
