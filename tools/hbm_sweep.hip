// HBM read-ceiling sweep (not part of the product): which access pattern
// streams a buffer far larger than the Infinity Cache fastest on this box.
// Variants: grid-stride vs one contiguous range per workgroup, loads in flight
// per lane, workgroups per CU, 256/512/1024-thread workgroups, nontemporal vs
// default policy, register loads vs LDS-DMA (global_load_lds_dwordx4).
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/hbm_sweep tools/hbm_sweep.hip && /tmp/hbm_sweep [GB]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}

// grid-stride: iteration i of block b reads U*T consecutive 16-B pieces at
// (i*grid + b)*U*T
template <int T, int U, bool NT>
__global__ void __launch_bounds__(T) k_stride(const u32x4* __restrict__ p, int64_t n16,
                                              uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const int64_t step = (int64_t)gridDim.x * T * U;
  for (int64_t i = (int64_t)blockIdx.x * T * U + threadIdx.x; i < n16; i += step) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = i + (int64_t)u * T;
      v[u] = j < n16 ? ld<NT>(p + j) : u32x4(0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// contiguous: block b owns pieces [b*per, (b+1)*per) and walks them with
// U*T pieces per iteration (what the scan does with its row range)
template <int T, int U, bool NT>
__global__ void __launch_bounds__(T) k_contig(const u32x4* __restrict__ p, int64_t n16,
                                              uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const int64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per;
  const int64_t hi = lo + per < n16 ? lo + per : n16;
  for (int64_t i = lo + threadIdx.x; i < hi; i += (int64_t)T * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = i + (int64_t)u * T;
      v[u] = j < hi ? ld<NT>(p + j) : u32x4(0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// contiguous per WAVE: wave w of the grid owns one range (the scan's wave
// ownership with U rows in flight)
template <int T, int U, bool NT>
__global__ void __launch_bounds__(T) k_wave(const u32x4* __restrict__ p, int64_t n16,
                                            uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const int64_t waves = (int64_t)gridDim.x * (T / 64);
  const int64_t w = (int64_t)blockIdx.x * (T / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t per = ((n16 + waves - 1) / waves + 63) / 64 * 64;
  const int64_t lo = w * per;
  const int64_t hi = lo + per < n16 ? lo + per : n16;
  for (int64_t i = lo + lane; i < hi; i += 64 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = i + (int64_t)u * 64;
      v[u] = j < hi ? ld<NT>(p + j) : u32x4(0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// the scan's pattern: 3 KB rows, 16 lanes per row (256 B per row per
// instruction, 4 rows per wave-instruction), U rows per lane group, block
// steps of 16U rows dealt round-robin over the grid; no arithmetic
template <int U>
__global__ void __launch_bounds__(256) k_rows(const u32x4* __restrict__ p, int64_t n16,
                                              uint32_t* __restrict__ out) {
  constexpr int S = 192;  // 16-B slots per 3 KB row
  const int64_t rows = n16 / S;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
  uint32_t acc = 0;
  for (int64_t r0 = (int64_t)blockIdx.x * 16 * U; r0 < rows; r0 += (int64_t)gridDim.x * 16 * U) {
    u32x4 v[U][12];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = r0 + wid * 4 * U + u * 4 + g;
#pragma unroll
      for (int c = 0; c < 12; ++c)
        v[u][c] = row < rows ? __builtin_nontemporal_load(p + row * S + c * 16 + j) : u32x4(0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < 12; ++c) acc ^= v[u][c][0] ^ v[u][c][1] ^ v[u][c][2] ^ v[u][c][3];
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// the same rows read as whole 1 KB wave-instructions (a wave's 4U rows are one
// contiguous run of 12U KB; lane L of instruction i reads bytes i KB + 16 L)
template <int U>
__global__ void __launch_bounds__(256) k_rows_flat(const u32x4* __restrict__ p, int64_t n16,
                                                   uint32_t* __restrict__ out) {
  constexpr int S = 192;
  const int64_t rows = n16 / S;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t acc = 0;
  for (int64_t r0 = (int64_t)blockIdx.x * 16 * U; r0 < rows; r0 += (int64_t)gridDim.x * 16 * U) {
    const int64_t w0 = (r0 + wid * 4 * U) * S;  // first 16-B slot of the wave's rows
    const int64_t lim = rows * S;
    u32x4 v[12 * U];
#pragma unroll
    for (int i = 0; i < 12 * U; ++i) {
      const int64_t q = w0 + i * 64 + lane;
      v[i] = q < lim ? __builtin_nontemporal_load(p + q) : u32x4(0);
    }
#pragma unroll
    for (int i = 0; i < 12 * U; ++i) acc ^= v[i][0] ^ v[i][1] ^ v[i][2] ^ v[i][3];
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// the batched filter's pattern: a block owns 256-row tiles (grid-stride over
// tiles) and reads them in K chunks of KB bytes per row (all 256 rows of the
// tile per chunk, rows 3 KB apart); 512 threads, two chunks in flight
template <int KB>
__global__ void __launch_bounds__(512) k_tile(const u32x4* __restrict__ p, int64_t n16,
                                              uint32_t* __restrict__ out) {
  constexpr int S = 192;             // 16-B slots per 3 KB row
  constexpr int C = KB / 16;         // lanes per row per chunk
  constexpr int P = 256 * C / 512;   // pieces per thread per chunk
  const int64_t tiles = n16 / (S * 256);
  const int t = threadIdx.x;
  uint32_t acc = 0;
  for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const u32x4* base = p + tile * 256 * S;
    for (int c = 0; c < S / C; c += 2) {
      u32x4 v[2][P];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < P; ++i) {
          const int row = (t / C) + i * (512 / C);
          v[h][i] = __builtin_nontemporal_load(base + row * S + (c + h) * C + t % C);
        }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < P; ++i) acc ^= v[h][i][0] ^ v[h][i][1] ^ v[h][i][2] ^ v[h][i][3];
    }
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

typedef __attribute__((address_space(3))) void* lds_ptr;

// LDS-DMA: each wave streams its contiguous range through a ring of S KB
// slots (1 KB per wave-instruction), counted vmcnt keeps S-1 in flight
template <int T, int S, int NT>
__global__ void __launch_bounds__(T) k_dma(const u32x4* __restrict__ p, int64_t n16,
                                           uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) u32x4 ring[T / 64][S][64];
  const int64_t waves = (int64_t)gridDim.x * (T / 64);
  const int wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * (T / 64) + wv;
  const int lane = threadIdx.x & 63;
  const int64_t per = ((n16 + waves - 1) / waves + 64 * S - 1) / (64 * S) * (64 * S);
  const int64_t lo = w * per;
  int64_t hi = lo + per < n16 ? lo + per : n16;
  if (hi < lo) hi = lo;
  const int64_t bytes = (hi - lo) * 16;
  const uint64_t base = reinterpret_cast<uint64_t>(p + lo);
  const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)base);
  const uint32_t bhi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  // one descriptor per 2 GB window
  uint32_t acc = 0;
  const int64_t iters = (hi - lo) / 64;
  for (int64_t it0 = 0; it0 < iters; it0 += S) {
    const uint64_t wb = (((uint64_t)bhi << 32) | blo) + (uint64_t)it0 * 1024;
    const int64_t left = bytes - it0 * 1024;
    const int nb = __builtin_amdgcn_readfirstlane((int)(left < (1ll << 30) ? left : (1ll << 30)));
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)wb, 0, nb, 0x00020000);
#pragma unroll
    for (int s = 0; s < S; ++s)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr)&ring[wv][s][0], 16,
                                               (uint32_t)(s * 1024 + lane * 16), 0, 0,
                                               NT ? 2 : 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const u32x4 v = ring[wv][s][lane];
      acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

typedef void (*Launch)(const u32x4*, int64_t, uint32_t*, int, hipStream_t);

template <template <int, int, bool> class K>
struct Dummy {};

static double run(const char* name, void (*fn)(const void*, int64_t, uint32_t*, int, hipStream_t),
                  const void* p, int64_t n16, uint32_t* out, int blocks, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  fn(p, n16, out, blocks, 0);  // warm
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(a, 0));
    fn(p, n16, out, blocks, 0);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  const double tbs = (double)n16 * 16 / (best * 1e-3) / 1e12;
  printf("%-34s blocks=%6d  %8.3f ms  %6.3f TB/s\n", name, blocks, best, tbs);
  fflush(stdout);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return tbs;
}

#define LAUNCHER(NAME, KERN, T, U, NT)                                                      \
  static void NAME(const void* p, int64_t n16, uint32_t* out, int blocks, hipStream_t s) { \
    hipLaunchKernelGGL((KERN<T, U, NT>), dim3(blocks), dim3(T), 0, s, (const u32x4*)p, n16, \
                       out);                                                                \
  }
#define ROWS(NAME, KERN, U)                                                                 \
  static void NAME(const void* p, int64_t n16, uint32_t* out, int blocks, hipStream_t s) { \
    hipLaunchKernelGGL((KERN<U>), dim3(blocks), dim3(256), 0, s, (const u32x4*)p, n16, out);  \
  }
#define TILE(NAME, KB)                                                                      \
  static void NAME(const void* p, int64_t n16, uint32_t* out, int blocks, hipStream_t s) { \
    hipLaunchKernelGGL((k_tile<KB>), dim3(blocks), dim3(512), 0, s, (const u32x4*)p, n16, out); \
  }
TILE(tile_128, 128)
TILE(tile_256, 256)
TILE(tile_512, 512)
ROWS(rows_1, k_rows, 1)
ROWS(rows_2, k_rows, 2)
ROWS(flat_1, k_rows_flat, 1)
ROWS(flat_2, k_rows_flat, 2)
LAUNCHER(stride_256_2_nt, k_stride, 256, 2, true)
LAUNCHER(stride_256_4_nt, k_stride, 256, 4, true)
LAUNCHER(stride_256_8_nt, k_stride, 256, 8, true)
LAUNCHER(stride_256_16_nt, k_stride, 256, 16, true)
LAUNCHER(stride_128_8_nt, k_stride, 128, 8, true)
LAUNCHER(stride_128_16_nt, k_stride, 128, 16, true)
LAUNCHER(stride_512_4_nt, k_stride, 512, 4, true)
LAUNCHER(stride_512_8_nt, k_stride, 512, 8, true)
LAUNCHER(stride_256_8_pl, k_stride, 256, 8, false)
LAUNCHER(wave_256_12_nt, k_wave, 256, 12, true)

int main(int argc, char** argv) {
  const double gb = argc > 1 ? atof(argv[1]) : 16.0;
  const int64_t bytes = (int64_t)(gb * 1e9) / 4096 * 4096;
  const int64_t n16 = bytes / 16;
  void* p = nullptr;
  uint32_t* out = nullptr;
  CHECK(hipMalloc(&p, bytes));
  CHECK(hipMalloc(&out, 1 << 20));
  CHECK(hipMemset(p, 1, bytes));
  CHECK(hipDeviceSynchronize());
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("buffer %.2f GB, %d CUs\n", bytes / 1e9, cus);
  const int reps = 5;
  struct V {
    const char* name;
    void (*fn)(const void*, int64_t, uint32_t*, int, hipStream_t);
    int threads;
  };
  const bool rows_only = getenv("HBM_SWEEP_ROWS") != nullptr;
  V rv[] = {
      {"tile 256 rows x 128 B chunks", tile_128, 512}, {"tile 256 rows x 256 B chunks", tile_256, 512},
      {"tile 256 rows x 512 B chunks", tile_512, 512},
      {"rows (scan pattern) U1", rows_1, 256}, {"rows (scan pattern) U2", rows_2, 256},
      {"rows flat 1 KB U1", flat_1, 256},      {"rows flat 1 KB U2", flat_2, 256},
      {"stride T256 U8 nt", stride_256_8_nt, 256},
  };
  V vs[] = {
      {"stride T256 U2 nt", stride_256_2_nt, 256},   {"stride T256 U4 nt", stride_256_4_nt, 256},
      {"stride T256 U8 nt", stride_256_8_nt, 256},   {"stride T256 U16 nt", stride_256_16_nt, 256},
      {"stride T128 U8 nt", stride_128_8_nt, 128},   {"stride T128 U16 nt", stride_128_16_nt, 128},
      {"stride T512 U4 nt", stride_512_4_nt, 512},   {"stride T512 U8 nt", stride_512_8_nt, 512},
      {"stride T256 U8 plain", stride_256_8_pl, 256}, {"wave T256 U12 nt", wave_256_12_nt, 256},
  };
  double best = 0;
  const char* bestn = "";
  int bestb = 0;
  const V* list = rows_only ? rv : vs;
  const int nlist = rows_only ? (int)(sizeof(rv) / sizeof(rv[0])) : (int)(sizeof(vs) / sizeof(vs[0]));
  for (int vi = 0; vi < nlist; ++vi) {
    const V& v = list[vi];
    for (int eighths : {4, 8, 12, 16, 24, 32}) {
      if (v.threads * eighths > 2048 * 8) continue;
      const double t = run(v.name, v.fn, p, n16, out, cus * eighths / 8, reps);
      if (t > best) {
        best = t;
        bestn = v.name;
        bestb = cus * eighths / 8;
      }
    }
  }
  printf("best: %s blocks=%d %.3f TB/s\n", bestn, bestb, best);
  CHECK(hipFree(p));
  CHECK(hipFree(out));
  return 0;
}
