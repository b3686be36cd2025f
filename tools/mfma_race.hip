// Does a VALU read of a v_mfma_i32_32x32x32_i8 result see the result after
// N wait states, under the traffic the filter kernels put beside it?
// (what the filter_img6_kernel pre-epilogue barrier fixes.)
//
// Each workgroup has 8 waves on one CU (two per SIMD).  Waves 0-3 ("probe")
// run `iters` times: one MFMA of A = all 1 (or all 2) bytes and B = all 1
// bytes with C = 0 into v[200:215], so every element is 32 (or 64,
// alternating), then N wait states, then a packed read of v[214:215] (the
// last registers, read as the epilogue's v_pk_fma_f32 reads them) and a
// 32-bit read of v200, all inside ONE asm statement (no compiler padding).
// A stale read shows the previous iteration's value.  Modes:
//   0  partner waves 4-7 exit at once
//   1  partner waves run a back-to-back MFMA chain meanwhile
//   2  partner waves stream 16-B loads from a 1 GiB buffer (VMEM returns
//      landing in their VGPRs on the same SIMD)
//   3  the probe itself has 4 16-B HBM loads in flight across its MFMA (their
//      returns land while the MFMA writes back), partners idle
//   4  modes 1 + 2 + 3 together
//
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_race.hip -o tools/mfma_race
//   ./tools/mfma_race [iters]
// prints one JSON line per (N, mode): stale elements / elements read.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr size_t kBufInts = (size_t)1 << 28;  // 1 GiB of int

__device__ __forceinline__ void partner(int iters, int mode, const i32x4* buf, unsigned* bad) {
  const bool mf = mode == 1 || mode == 4, ld = mode == 2 || mode == 4;
  if (!mf && !ld) return;
  const i32x4 a = {0x01010101, 0x01010101, 0x01010101, 0x01010101};
  i32x16 acc = i32x16(0);
  i32x4 x = i32x4(0);
  const size_t n4 = kBufInts / 4;
  size_t p = ((size_t)blockIdx.x * 256 + (threadIdx.x & 255)) * 977;
  for (int i = 0; i < iters * 4; ++i) {
    if (ld) {
      p = (p + 256 * 4099) % n4;
      x ^= __builtin_nontemporal_load(buf + p);
    }
    if (mf) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, acc, 0, 0, 0);
  }
  if (acc[0] == 0x7fffffff || x[0] == 0x7fffffff) atomicAdd(bad + 1, 1u);
}

#define RACE_KERNEL(N, NOPS)                                                                      \
  __global__ void __launch_bounds__(512, 1)                                                       \
      race_##N(int iters, int mode, const i32x4* buf, unsigned* bad) {                            \
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);                              \
    if (w >= 4) {                                                                                 \
      partner(iters, mode, buf, bad);                                                             \
      return;                                                                                     \
    }                                                                                             \
    unsigned nbad = 0;                                                                            \
    const i32x4 b = {0x01010101, 0x01010101, 0x01010101, 0x01010101};                             \
    const size_t n4 = kBufInts / 4;                                                               \
    size_t p = ((size_t)blockIdx.x * 256 + threadIdx.x) * 1237 + 1;                               \
    i32x4 sink = i32x4(0);                                                                        \
    for (int i = 0; i < iters; ++i) {                                                             \
      const int v = (i & 1) ? 0x02020202 : 0x01010101;                                            \
      const i32x4 a = {v, v, v, v};                                                               \
      i32x4 l0 = i32x4(0), l1 = l0, l2 = l0, l3 = l0;                                             \
      if (mode >= 3) {                                                                            \
        p = (p + 256 * 8191) % (n4 - 4);                                                          \
        l0 = __builtin_nontemporal_load(buf + p);                                                 \
        l1 = __builtin_nontemporal_load(buf + p + 1);                                             \
        l2 = __builtin_nontemporal_load(buf + p + 2);                                             \
        l3 = __builtin_nontemporal_load(buf + p + 3);                                             \
      }                                                                                           \
      f32x2 hi;                                                                                   \
      int lo;                                                                                     \
      asm volatile(                                                                               \
          "s_nop 4\n\tv_mfma_i32_32x32x32_i8 v[200:215], %2, %3, 0\n\t" NOPS                      \
          "v_pk_add_f32 %0, v[214:215], 0\n\tv_mov_b32 %1, v200\n\ts_nop 1"                       \
          : "=&v"(hi), "=&v"(lo)                                                                  \
          : "v"(a), "v"(b)                                                                        \
          : "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209",      \
            "v210", "v211", "v212", "v213", "v214", "v215");                                      \
      const int expect = (i & 1) ? 64 : 32;                                                       \
      const float fe = __int_as_float(expect);                                                    \
      nbad += (hi[0] != fe) + (hi[1] != fe) + (lo != expect);                                     \
      sink ^= l0 ^ l1 ^ l2 ^ l3;                                                                  \
    }                                                                                             \
    atomicAdd(bad, nbad);                                                                         \
    if (sink[0] == 0x7fffffff) atomicAdd(bad + 1, 1u);                                            \
  }

#define S15 "s_nop 15\n\t"
RACE_KERNEL(2, "s_nop 1\n\t")
RACE_KERNEL(4, "s_nop 3\n\t")
RACE_KERNEL(8, "s_nop 7\n\t")
RACE_KERNEL(12, "s_nop 11\n\t")
RACE_KERNEL(16, S15)
RACE_KERNEL(24, S15 "s_nop 7\n\t")
RACE_KERNEL(41, S15 S15 "s_nop 8\n\t")

typedef void (*Fn)(int, int, const i32x4*, unsigned*);

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
  unsigned* bad = nullptr;
  i32x4* buf = nullptr;
  if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&buf, kBufInts * 4) != hipSuccess) return 1;
  if (hipMemset(buf, 1, kBufInts * 4) != hipSuccess) return 1;
  const struct {
    int n;
    Fn f;
  } ks[] = {{2, race_2}, {4, race_4}, {8, race_8}, {12, race_12}, {16, race_16}, {24, race_24},
            {41, race_41}};
  for (const auto& k : ks) {
    for (int mode = 0; mode < 5; ++mode) {
      if (hipMemset(bad, 0, 8) != hipSuccess) return 1;
      hipLaunchKernelGGL(k.f, dim3(cus), dim3(512), 0, 0, iters, mode, buf, bad);
      if (hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "kernel failed\n");
        return 1;
      }
      unsigned h[2] = {0, 0};
      if (hipMemcpy(h, bad, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
      const double read = (double)cus * 4 * 64 * 3 * iters;
      printf("{\"wait_states\": %d, \"mode\": %d, \"stale\": %u, \"read\": %.0f}\n", k.n, mode,
             h[0], read);
      fflush(stdout);
    }
  }
  return 0;
}
