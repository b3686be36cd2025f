// Coded (multi-codebook) index on gfx950.
//
// The reference's coder (src/fenix/io/coder/coder.py) keeps `num_codebooks`
// (nb) independent codebooks of `codebook_size` (ks) full-width codewords.  A
// row's code is the composite  sum_j argmin_c dist(x, C_j[c]) * ks^(nb-1-j)
// (coder.py:171-186 with maxval = 1, which is how index.make encodes a table,
// index.py:46-49); the codebooks are trained by mini-batch k-means
// (coder.py:53-65 under torch.vmap, 94-118); a probe search keeps the rows whose
// code is among the `probes` composites nearest to the target (index.py:113-126).
//
//   assign_kernel    nearest codeword per (row, codebook).  An fp32 MFMA GEMM of
//                    128-row x 256-codeword tiles (the batched search's tiling,
//                    knn_batch.hip; f16 rows are widened while staging to LDS)
//                    whose epilogue turns each dot product into the metric's
//                    distance, min-reduces 64-bit (order_key(dist) << 32 | index)
//                    keys over each codebook segment in registers and lane
//                    shuffles, and issues one atomicMin per (row, codebook, wave).
//                    Ties go to the lowest codeword index.
//   finalize_kernel  keys -> codeword index, composite code, distance.
//   update_kernel    k-means step: codeword <- mean(codeword, assigned rows)
//                    (torch.index_reduce(..., "mean") keeps the codeword itself
//                    in the mean, coder.py:60), summed in row order in LDS:
//                    deterministic, no float atomics.
//   composite_kernel composite scores of a target, then a segmented radix sort
//                    (hipcub) of (score, code) keys -> the probe set.
//   mask_kernel      row bitmap = (row code in the probe set) AND filter bitmap,
//                    consumed by the ordinary masked scan, which skips the loads
//                    of masked-out rows.
#include <hipcub/hipcub.hpp>
#include <stdlib.h>

#include "fx_internal.h"
#include "fx_wave.h"

namespace fx {

namespace {

constexpr int kCM = 128;         // rows per tile
constexpr int kCQ = 256;         // codeword slots per block
constexpr int kCK = 32;          // K chunk
constexpr int kCLds = kCK + 4;   // padded LDS row (floats)
constexpr int kCThreads = 512;   // 8 waves: 4 row groups x 2 slot halves
constexpr int kCTiles = 4;       // 32-slot MFMA tiles per wave

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

struct AssignShared {
  float xs[2][kCM * kCLds];
  float ws[2][kCQ * kCLds];
  float xnorm[kCM];
};

struct AssignArgs {
  const void* X;     // group g reads rows [g*rows, (g+1)*rows) of a [.][d] matrix
  int64_t rows;      // rows per group
  int d;
  int vec;           // rows 16-B (f32) / 8-B (f16) aligned and d % 4 == 0
  const float* W;    // padded codewords [groups][slots][d4]
  const float* wn;   // per slot: ||w||^2 (L2), max(||w||, eps) (cosine)
  int d4;            // d rounded up to 4
  int slots;         // slots per group = nbg * ks_pad
  int nbg, ks, ks_pad;
  int64_t num_tiles;
  uint64_t* keys;    // [groups][rows][nbg]
};

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

template <typename T>
__device__ __forceinline__ f32x4 x_piece(const T* X, int64_t gr, int d, int k, int vec) {
  const T* p = X + gr * (int64_t)d + k;
  if (vec) {
    if constexpr (sizeof(T) == 4) {
      return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    } else {
      const u32x2 u = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
      const f16x4 hv = __builtin_bit_cast(f16x4, u);
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (float)hv[e];
      return v;
    }
  }
  f32x4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = (k + e < d) ? (float)p[e] : 0.f;
  return v;
}

struct CPrefetch {
  f32x4 x[kCM * 8 / kCThreads];
  f32x4 w[kCQ * 8 / kCThreads];
};

template <typename T>
__device__ __forceinline__ void cprefetch(CPrefetch& p, const AssignArgs& a, const T* X,
                                          const float* W, int64_t r0, int s0, int k0, int tid) {
#pragma unroll
  for (int i = 0; i < kCM * 8 / kCThreads; ++i) {
    const int idx = i * kCThreads + tid;  // row = idx/8, col4 = idx%8
    const int64_t gr = r0 + (idx >> 3);
    const int k = k0 + (idx & 7) * 4;
    p.x[i] = (gr < a.rows && k < a.d) ? x_piece(X, gr, a.d, k, a.vec) : f32x4(0.f);
  }
#pragma unroll
  for (int i = 0; i < kCQ * 8 / kCThreads; ++i) {
    const int idx = i * kCThreads + tid;
    const int gs = s0 + (idx >> 3);
    const int k = k0 + (idx & 7) * 4;
    p.w[i] = (gs < a.slots && k < a.d4) ? ld4(W + (int64_t)gs * a.d4 + k) : f32x4(0.f);
  }
}

__device__ __forceinline__ void cstore(const CPrefetch& p, AssignShared* sh, int buf, int tid) {
#pragma unroll
  for (int i = 0; i < kCM * 8 / kCThreads; ++i) {
    const int idx = i * kCThreads + tid;
    *reinterpret_cast<f32x4*>(&sh->xs[buf][(idx >> 3) * kCLds + (idx & 7) * 4]) = p.x[i];
  }
#pragma unroll
  for (int i = 0; i < kCQ * 8 / kCThreads; ++i) {
    const int idx = i * kCThreads + tid;
    *reinterpret_cast<f32x4*>(&sh->ws[buf][(idx >> 3) * kCLds + (idx & 7) * 4]) = p.w[i];
  }
}

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// min over the 32 lanes of a half-wave (every lane must execute it)
__device__ __forceinline__ uint64_t half_min(uint64_t v, int width) {
  for (int m = 1; m < width; m <<= 1) v = umin64(v, shfl_xor_u64(v, m));
  return v;
}

template <typename T, int METRIC>
__global__ void __launch_bounds__(kCThreads, 1) assign_kernel(AssignArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  AssignShared* sh = reinterpret_cast<AssignShared*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int rg = wid & 3;
  const int qtile0 = (wid >> 2) * kCTiles;
  const int h = lane >> 5, l32 = lane & 31;
  const int g = blockIdx.z;
  const T* X = reinterpret_cast<const T*>(a.X) + (int64_t)g * a.rows * a.d;
  const float* W = a.W + (int64_t)g * a.slots * a.d4;
  const float* wn = a.wn + (int64_t)g * a.slots;
  uint64_t* keys = a.keys + (int64_t)g * a.rows * a.nbg;
  const int s0 = blockIdx.y * kCQ;
  const int nchunks = (a.d4 + kCK - 1) / kCK;

  float wnr[kCTiles];
  int cbs[kCTiles], locs[kCTiles];
  bool sv[kCTiles];
#pragma unroll
  for (int qt = 0; qt < kCTiles; ++qt) {
    const int slot = s0 + (qtile0 + qt) * 32 + l32;
    cbs[qt] = slot / a.ks_pad;
    locs[qt] = slot - cbs[qt] * a.ks_pad;
    sv[qt] = slot < a.slots && locs[qt] < a.ks;
    wnr[qt] = sv[qt] ? wn[slot] : 1.f;
  }

  for (int64_t ti = blockIdx.x; ti < a.num_tiles; ti += gridDim.x) {
    const int64_t r0 = ti * kCM;
    f32x16 acc[kCTiles];
#pragma unroll
    for (int qt = 0; qt < kCTiles; ++qt) acc[qt] = f32x16(0.f);
    float sumsq = 0.f;

    CPrefetch pf;
    cprefetch<T>(pf, a, X, W, r0, s0, 0, tid);
    __syncthreads();  // the previous tile's epilogue is done with the LDS
    cstore(pf, sh, 0, tid);
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
      const int buf = c & 1;
      if (c + 1 < nchunks) cprefetch<T>(pf, a, X, W, r0, s0, (c + 1) * kCK, tid);
      const float* xs = sh->xs[buf] + (rg * 32 + l32) * kCLds + 4 * h;
      const float* ws = sh->ws[buf] + (qtile0 * 32 + l32) * kCLds + 4 * h;
#pragma unroll
      for (int gg = 0; gg < kCK / 8; ++gg) {
        const f32x4 av = ld4(xs + 8 * gg);
        if constexpr (METRIC != 1) {
#pragma unroll
          for (int t = 0; t < 4; ++t) sumsq = fmaf(av[t], av[t], sumsq);
        }
#pragma unroll
        for (int qt = 0; qt < kCTiles; ++qt) {
          const f32x4 bv = ld4(ws + qt * 32 * kCLds + 8 * gg);
#pragma unroll
          for (int t = 0; t < 4; ++t)
            acc[qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[t], bv[t], acc[qt], 0, 0, 0);
        }
      }
      if (c + 1 < nchunks) cstore(pf, sh, buf ^ 1, tid);
      __syncthreads();
    }

    if constexpr (METRIC != 1) {
      sumsq += __shfl_xor(sumsq, 32);
      if (h == 0 && qtile0 == 0) sh->xnorm[rg * 32 + l32] = sumsq;
    }
    __syncthreads();

#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int lr = rg * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int64_t row = r0 + lr;
      const bool ok = row < a.rows;
      float xn = 0.f;
      if constexpr (METRIC != 1) xn = sh->xnorm[lr];
      uint64_t run = kEmpty;
      int run_cb = -1;
#pragma unroll
      for (int qt = 0; qt < kCTiles; ++qt) {
        const float dot = acc[qt][r];
        float dist;
        if constexpr (METRIC == 0) {
          dist = fmaxf(xn + wnr[qt] - 2.f * dot, 0.f);  // squared: same argmin
        } else if constexpr (METRIC == 1) {
          dist = -dot;
        } else {
          dist = 0.5f - 0.5f * (dot / (fmaxf(sqrtf(xn), 1e-12f) * wnr[qt]));
        }
        uint64_t key = sv[qt] ? make_comp(dist, (uint32_t)locs[qt]) : kEmpty;
        if (a.ks_pad >= 32) {
          // the 32-slot tile lies inside one codebook (wave-uniform branch)
          if (cbs[qt] != run_cb) {
            if (run_cb >= 0) {
              const uint64_t m = half_min(run, 32);
              if (l32 == 0 && ok && m != kEmpty && run_cb < a.nbg)
                atomicMin(reinterpret_cast<unsigned long long*>(&keys[row * a.nbg + run_cb]),
                          (unsigned long long)m);
            }
            run = key;
            run_cb = cbs[qt];
          } else {
            run = umin64(run, key);
          }
        } else {
          key = half_min(key, a.ks_pad);  // aligned segments of ks_pad lanes
          if (ok && locs[qt] == 0 && key != kEmpty && cbs[qt] < a.nbg)
            atomicMin(reinterpret_cast<unsigned long long*>(&keys[row * a.nbg + cbs[qt]]),
                      (unsigned long long)key);
        }
      }
      if (a.ks_pad >= 32 && run_cb >= 0) {
        const uint64_t m = half_min(run, 32);
        if (l32 == 0 && ok && m != kEmpty && run_cb < a.nbg)
          atomicMin(reinterpret_cast<unsigned long long*>(&keys[row * a.nbg + run_cb]),
                    (unsigned long long)m);
      }
    }
  }
}

// pack codewords into [groups][slots][d4] (zero padding) + per-slot norm term
__global__ void pack_kernel(const float* __restrict__ cw, int64_t groups, int nbg, int ks,
                            int ks_pad, int d, int d4, int metric, float* __restrict__ W,
                            float* __restrict__ wn) {
  const int64_t slot = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t slots = (int64_t)nbg * ks_pad;
  if (slot >= groups * slots) return;
  const int64_t g = slot / slots;
  const int s = (int)(slot - g * slots);
  const int cb = s / ks_pad, loc = s - cb * ks_pad;
  const bool valid = loc < ks;
  const float* src = cw + (((g * nbg) + cb) * ks + loc) * (int64_t)d;
  float sq = 0.f;
  for (int i = lane; i < d4; i += 64) {
    const float v = (valid && i < d) ? src[i] : 0.f;
    W[slot * d4 + i] = v;
    sq = fmaf(v, v, sq);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) sq += __shfl_xor(sq, m);
  if (lane == 0) wn[slot] = metric == FX_METRIC_COS ? fmaxf(sqrtf(sq), 1e-12f) : sq;
}

__global__ void finalize_kernel(const uint64_t* __restrict__ keys, int64_t n, int nb, int ks,
                                int metric, int32_t* __restrict__ out_index,
                                int64_t* __restrict__ out_code, float* __restrict__ out_dist) {
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n) return;
  int64_t code = 0;
  for (int j = 0; j < nb; ++j) {
    const uint64_t key = keys[row * nb + j];
    const int32_t loc = key == kEmpty ? -1 : (int32_t)(key & 0xffffffffull);
    if (out_index) out_index[row * nb + j] = loc;
    code = code * ks + (loc < 0 ? 0 : loc);
    if (out_dist) {
      float f = key == kEmpty ? __builtin_nanf("") : key_float((uint32_t)(key >> 32));
      if (metric == FX_METRIC_L2) f = sqrtf(f);
      out_dist[row * nb + j] = f;
    }
  }
  if (out_code) out_code[row] = code;
}

// one wave per row: mode 0 -> sum of squares, mode 1 -> max(||x||, eps)
template <typename T>
__global__ void rownorm_kernel(const T* __restrict__ X, int64_t n, int d, int mode,
                               float* __restrict__ out) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const T* p = X + row * (int64_t)d;
  float s = 0.f;
  for (int i = lane; i < d; i += 64) {
    const float v = (float)p[i];
    s = fmaf(v, v, s);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  if (lane == 0) out[row] = mode == 0 ? s : fmaxf(sqrtf(s), 1e-12f);
}

// F.normalize in place (coder.py:55-56): x / max(||x||, 1e-12), one wave per row
__global__ void normalize_kernel(float* __restrict__ X, int64_t n, int d) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  float* p = X + row * (int64_t)d;
  float s = 0.f;
  for (int i = lane; i < d; i += 64) s = fmaf(p[i], p[i], s);
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  const float nrm = fmaxf(sqrtf(s), 1e-12f);
  for (int i = lane; i < d; i += 64) p[i] = p[i] / nrm;
}

// k-means codeword update (coder.py:59-63): block (c, j) averages codeword c of
// codebook j with the sample rows assigned to it.  1024 threads; thread t owns
// dims t, t+1024, ... in registers (d <= 16384); each 1024-entry slice of the
// assignments is compacted in LDS (ballot, row order) and its rows are summed
// four at a time (independent loads in flight).  The order of the sum is fixed:
// deterministic, no float atomics.
constexpr int kUpdThreads = 1024;
constexpr int kUpdDims = 16;  // registers per thread: d <= 16 * 1024

template <typename T>
__global__ void __launch_bounds__(kUpdThreads) update_kernel(const T* __restrict__ X, int64_t bs,
                                                             int d,
                                                             const int32_t* __restrict__ assign,
                                                             const float* __restrict__ rnorm,
                                                             float* __restrict__ W, int ks,
                                                             int cosine) {
  __shared__ int list[kUpdThreads];
  __shared__ int wcount[16];
  __shared__ float red[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int c = blockIdx.x, j = blockIdx.y;
  float* w = W + ((int64_t)j * ks + c) * d;
  const T* Xj = X + (int64_t)j * bs * d;
  const int32_t* as = assign + (int64_t)j * bs;
  const float* rn = rnorm ? rnorm + (int64_t)j * bs : nullptr;
  float acc[kUpdDims];
#pragma unroll
  for (int u = 0; u < kUpdDims; ++u) {
    const int dim = tid + u * kUpdThreads;
    acc[u] = dim < d ? w[dim] : 0.f;  // include_self
  }
  int count = 1;
  const uint64_t ltmask = (1ull << lane) - 1ull;
  for (int64_t i0 = 0; i0 < bs; i0 += kUpdThreads) {
    const int64_t i = i0 + tid;
    const bool m = i < bs && as[i] == c;
    const uint64_t b = __ballot(m);
    if (lane == 0) wcount[wid] = __popcll(b);
    __syncthreads();
    int base = 0, total = 0;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      base += v < wid ? wcount[v] : 0;
      total += wcount[v];
    }
    if (m) list[base + __popcll(b & ltmask)] = (int)(i - i0);
    __syncthreads();
    for (int e0 = 0; e0 < total; e0 += 4) {
      const T* xr[4];
      float sc[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int e = e0 + t < total ? e0 + t : e0;
        const int64_t r = i0 + list[e];
        xr[t] = Xj + r * d;
        sc[t] = (e0 + t < total) ? 1.f : 0.f;
        if (cosine && e0 + t < total) sc[t] = rn[r];
      }
#pragma unroll
      for (int u = 0; u < kUpdDims; ++u) {
        const int dim = tid + u * kUpdThreads;
        if (dim < d) {
          float v[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] = (float)xr[t][dim];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            if (e0 + t < total) acc[u] += cosine ? v[t] / sc[t] : v[t];
          }
        }
      }
    }
    count += total;
    __syncthreads();
  }
  float sq = 0.f;
#pragma unroll
  for (int u = 0; u < kUpdDims; ++u) {
    acc[u] = acc[u] / (float)count;
    if (tid + u * kUpdThreads < d) sq = fmaf(acc[u], acc[u], sq);
  }
  float nrm = 1.f;
  if (cosine) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) sq += __shfl_xor(sq, m);
    if (lane == 0) red[wid] = sq;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int v = 0; v < 16; ++v) t += red[v];
    nrm = fmaxf(sqrtf(t), 1e-12f);
  }
#pragma unroll
  for (int u = 0; u < kUpdDims; ++u) {
    const int dim = tid + u * kUpdThreads;
    if (dim < d) w[dim] = cosine ? acc[u] / nrm : acc[u];
  }
}

__global__ void offsets_kernel(int* off, int64_t nq, int64_t C) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= nq) off[i] = (int)(i * C);
}

__global__ void emit_kernel(const uint64_t* __restrict__ sorted, int64_t C, int64_t p,
                            int64_t* __restrict__ out_code, float* __restrict__ out_score,
                            uint32_t* __restrict__ sel, int64_t words) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t q = blockIdx.y;
  if (i >= p) return;
  const uint64_t key = sorted[q * C + i];
  const int64_t code = (int64_t)(key & 0xffffffffull);
  if (out_code) out_code[q * p + i] = code;
  if (out_score) out_score[q * p + i] = key_float((uint32_t)(key >> 32));
  if (sel) atomicOr(&sel[q * words + (code >> 5)], 1u << (code & 31));
}

// grid-stride over rows; one count atomic per block (a per-wave atomic on one
// address serialised the kernel: 340 us for 10M rows)
__global__ void __launch_bounds__(256) mask_kernel(const int64_t* __restrict__ code, int64_t n,
                                                   const uint32_t* __restrict__ sel, int64_t ncodes,
                                                   const uint32_t* __restrict__ filter,
                                                   uint32_t* __restrict__ out, int64_t words,
                                                   unsigned long long* __restrict__ count) {
  __shared__ unsigned int wsum[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned int kept = 0;
  for (int64_t base = (int64_t)blockIdx.x * 256; base < n; base += (int64_t)gridDim.x * 256) {
    const int64_t row = base + threadIdx.x;
    bool bit = false;
    if (row < n) {
      const int64_t c = code[row];
      bit = c >= 0 && c < ncodes && ((sel[c >> 5] >> (c & 31)) & 1u);
      if (filter != nullptr) bit = bit && ((filter[row >> 5] >> (row & 31)) & 1u);
    }
    const uint64_t b = __ballot(bit);
    const int64_t w0 = (row - lane) >> 5;
    if (lane == 0 && w0 < words) out[w0] = (uint32_t)b;
    if (lane == 32 && w0 + 1 < words) out[w0 + 1] = (uint32_t)(b >> 32);
    kept += (unsigned int)__popcll(b);
  }
  if (count == nullptr) return;
  if (lane == 0) wsum[wid] = kept;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int t = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (t) atomicAdd(count, (unsigned long long)t);
  }
}

// ---- ordered bitmap -> row list compaction (three passes, no atomics)
constexpr int kCompactWords = 2048;  // words (65 536 rows) per block

__global__ void __launch_bounds__(256) compact_count_kernel(const uint32_t* __restrict__ mask,
                                                            int64_t words,
                                                            uint32_t* __restrict__ block_count) {
  __shared__ unsigned int wsum[4];
  const int64_t w0 = (int64_t)blockIdx.x * kCompactWords;
  unsigned int c = 0;
  for (int i = threadIdx.x; i < kCompactWords; i += 256)
    if (w0 + i < words) c += __popc(mask[w0 + i]);
  for (int m = 32; m >= 1; m >>= 1) c += __shfl_xor(c, m);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) block_count[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// one 1024-thread block: exclusive scan of the block counts (in place), total
__global__ void __launch_bounds__(1024) compact_scan_kernel(uint32_t* __restrict__ v, int64_t nb,
                                                            unsigned long long* __restrict__ total) {
  __shared__ unsigned int wsum[16];
  __shared__ unsigned int carry;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < nb; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const unsigned int x = i < nb ? v[i] : 0u;
    const unsigned int incl = wave_incl_scan(x, lane);
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    unsigned int before = carry;
    for (int w = 0; w < wid; ++w) before += wsum[w];
    if (i < nb) v[i] = before + incl - x;
    __syncthreads();
    if (threadIdx.x == 1023) carry = before + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0 && total != nullptr) *total = carry;
}

// each thread owns 8 consecutive words; block scan of thread sums gives offsets
__global__ void __launch_bounds__(256) compact_write_kernel(const uint32_t* __restrict__ mask,
                                                            int64_t words,
                                                            const uint32_t* __restrict__ offs,
                                                            int32_t* __restrict__ rows) {
  __shared__ unsigned int wsum[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t w0 = (int64_t)blockIdx.x * kCompactWords + threadIdx.x * 8;
  uint32_t m[8];
  unsigned int c = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m[j] = (w0 + j < words) ? mask[w0 + j] : 0u;
    c += __popc(m[j]);
  }
  const unsigned int incl = wave_incl_scan(c, lane);
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  unsigned int pos = offs[blockIdx.x] + incl - c;
  for (int w = 0; w < wid; ++w) pos += wsum[w];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t bits = m[j];
    while (bits) {
      const int b = __ffs(bits) - 1;
      rows[pos++] = (int32_t)((w0 + j) * 32 + b);
      bits &= bits - 1;
    }
  }
}

// probe codes from the merged (score, code) lists -> selected-code bitmap
__global__ void sel_kernel(const int64_t* __restrict__ codes, int64_t p, uint32_t* __restrict__ sel,
                           int64_t words) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t q = blockIdx.y;
  if (i >= p) return;
  const int64_t c = codes[q * p + i];
  if (c >= 0) atomicOr(&sel[q * words + (c >> 5)], 1u << (c & 31));
}

// composite keys as [nq][nlists][kin] lists for the merge kernels (kEmpty pad)
__global__ void composite_lists_kernel(const float* __restrict__ dist, int nb, int ks, int64_t C,
                                       int64_t padded, uint64_t* __restrict__ keys) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t q = blockIdx.y;
  if (c >= padded) return;
  if (c >= C) {
    keys[q * padded + c] = kEmpty;
    return;
  }
  int digit[32];
  int64_t rem = c;
  for (int j = nb - 1; j >= 0; --j) {
    digit[j] = (int)(rem % ks);
    rem /= ks;
  }
  const float* dq = dist + q * (int64_t)nb * ks;
  float s = 0.f;
  for (int j = 0; j < nb; ++j) s = s + dq[j * ks + digit[j]];
  keys[q * padded + c] = make_comp(s, (uint32_t)c);
}

size_t align256(size_t v) { return (v + 255) / 256 * 256; }

int pad_ks(int64_t ks) {
  if (ks >= 32) return (int)((ks + 31) / 32 * 32);
  int p = 1;
  while (p < ks) p <<= 1;
  return p;
}

struct AssignLayout {
  int ks_pad, d4, slots;
  size_t off_w, off_wn, off_keys, total;
};

AssignLayout assign_layout(int64_t groups, int64_t rows, int64_t nbg, int64_t ks, int64_t d) {
  AssignLayout l;
  l.ks_pad = pad_ks(ks);
  l.d4 = (int)((d + 3) / 4 * 4);
  l.slots = (int)(nbg * l.ks_pad);
  size_t off = 0;
  l.off_w = off;
  off += align256((size_t)groups * l.slots * l.d4 * 4);
  l.off_wn = off;
  off += align256((size_t)groups * l.slots * 4);
  l.off_keys = off;
  off += align256((size_t)groups * rows * nbg * 8);
  l.total = off;
  return l;
}

template <typename T, int METRIC>
void* assign_fn() {
  return (void*)assign_kernel<T, METRIC>;
}

int run_assign(const void* X, int dtype, int64_t groups, int64_t rows, int64_t d,
               const float* cw, int64_t nbg, int64_t ks, int metric, char* ws,
               const AssignLayout& l, hipStream_t st) {
  float* W = reinterpret_cast<float*>(ws + l.off_w);
  float* wn = reinterpret_cast<float*>(ws + l.off_wn);
  uint64_t* keys = reinterpret_cast<uint64_t*>(ws + l.off_keys);
  const int64_t nslots = groups * l.slots;
  hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((nslots + 3) / 4)), dim3(256), 0, st, cw, groups,
                     (int)nbg, (int)ks, l.ks_pad, (int)d, l.d4, metric, W, wn);
  int rc = check_launch("pack_kernel");
  if (rc) return rc;
  hipError_t e = hipMemsetAsync(keys, 0xFF, (size_t)groups * rows * nbg * 8, st);
  if (e != hipSuccess) {
    set_error("assign memset: %s", hipGetErrorString(e));
    return FX_EHIP;
  }
  if (rows == 0) return FX_OK;
  AssignArgs a = {};
  a.X = X;
  a.rows = rows;
  a.d = (int)d;
  const size_t esz = dtype == FX_DTYPE_F32 ? 4 : 2;
  a.vec = (d % 4 == 0) && ((uintptr_t)X % (4 * esz) == 0);
  a.W = W;
  a.wn = wn;
  a.d4 = l.d4;
  a.slots = l.slots;
  a.nbg = (int)nbg;
  a.ks = (int)ks;
  a.ks_pad = l.ks_pad;
  a.num_tiles = (rows + kCM - 1) / kCM;
  a.keys = keys;
  void* fn;
  if (dtype == FX_DTYPE_F32) {
    fn = metric == FX_METRIC_L2 ? assign_fn<float, 0>()
         : metric == FX_METRIC_IP ? assign_fn<float, 1>() : assign_fn<float, 2>();
  } else {
    fn = metric == FX_METRIC_L2 ? assign_fn<_Float16, 0>()
         : metric == FX_METRIC_IP ? assign_fn<_Float16, 1>() : assign_fn<_Float16, 2>();
  }
  const size_t smem = sizeof(AssignShared);
  if (int rc2 = allow_lds((const void*)fn)) return rc2;
  int cus = 0;
  rc = device_cus(&cus);
  if (rc) return rc;
  const int64_t ytiles = (l.slots + kCQ - 1) / kCQ;
  int64_t bx = a.num_tiles < cus ? a.num_tiles : cus;
  if (ytiles > 65535 || groups > 65535) {
    set_error("coded index too large: %lld slot tiles, %lld groups", (long long)ytiles,
              (long long)groups);
    return FX_EUNSUPPORTED;
  }
  void* args[] = {(void*)&a};
  e = hipLaunchKernel(fn, dim3((unsigned)bx, (unsigned)ytiles, (unsigned)groups), dim3(kCThreads),
                      args, smem, st);
  if (e != hipSuccess) {
    set_error("assign_kernel launch: %s", hipGetErrorString(e));
    return FX_EHIP;
  }
  return check_launch("assign_kernel");
}

int validate_code(int64_t n, int64_t d, int dtype, int64_t nb, int64_t ks, int metric) {
  if (n < 0 || d <= 0 || d > (1 << 20)) {
    set_error("invalid shape n=%lld d=%lld", (long long)n, (long long)d);
    return FX_EINVAL;
  }
  if (dtype != FX_DTYPE_F32 && dtype != FX_DTYPE_F16) {
    set_error("unsupported dtype %d", dtype);
    return FX_EINVAL;
  }
  if (metric != FX_METRIC_L2 && metric != FX_METRIC_IP && metric != FX_METRIC_COS) {
    set_error("unknown metric %d", metric);
    return FX_EINVAL;
  }
  if (nb <= 0 || ks <= 0) {
    set_error("invalid coding: num_codebooks=%lld codebook_size=%lld", (long long)nb,
              (long long)ks);
    return FX_EINVAL;
  }
  return FX_OK;
}

// ks^nb, or -1 above 2^31 - 1
int64_t composite_count(int64_t nb, int64_t ks) {
  int64_t c = 1;
  for (int64_t j = 0; j < nb; ++j) {
    if (c > ((int64_t)1 << 31) / ks) return -1;
    c *= ks;
  }
  return c < ((int64_t)1 << 31) ? c : -1;
}

constexpr int64_t kProbeMerge = 4096;  // probes up to this go through the merge kernels

struct ProbeLayout {
  int64_t C, kin, nlists, padded, pmax;
  size_t temp_bytes, merge_bytes;
  size_t off_keys, off_sorted, off_off, off_temp, off_merge, off_codes, off_scores, total;
};

// composite scores of coder.call (coder.py:171-181): probes <= 4096 are
// selected by the merge kernels (keys viewed as lists of kin), larger probe
// sets (and the full argsort of maxval=None) by a segmented radix sort.
int probe_layout(int64_t nq, int64_t nb, int64_t ks, ProbeLayout* p) {
  p->C = composite_count(nb, ks);
  if (p->C < 0 || nq * p->C >= ((int64_t)1 << 31) || nb > 32) {
    set_error("composite code space %lld^%lld x %lld queries exceeds 2^31", (long long)ks,
              (long long)nb, (long long)nq);
    return FX_EUNSUPPORTED;
  }
  p->kin = p->C < kProbeMerge ? p->C : kProbeMerge;
  p->nlists = (p->C + p->kin - 1) / p->kin;
  p->padded = p->nlists * p->kin;
  p->pmax = p->C < kProbeMerge ? p->C : kProbeMerge;
  MergePlan mp;
  int rc = plan_merge(nq, p->nlists, p->kin, p->pmax, &mp);
  if (rc) return rc;
  p->merge_bytes = mp.ws_bytes;
  p->temp_bytes = 0;
  hipError_t e = hipcub::DeviceSegmentedRadixSort::SortKeys(
      nullptr, p->temp_bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)(nq * p->C),
      (int)nq, (const int*)nullptr, (const int*)nullptr, 0, 64, (hipStream_t)0);
  if (e != hipSuccess) {
    set_error("segmented sort sizing: %s", hipGetErrorString(e));
    return FX_EHIP;
  }
  size_t off = 0;
  p->off_keys = off;
  off += align256((size_t)nq * p->padded * 8);
  p->off_sorted = off;
  off += align256((size_t)nq * p->C * 8);
  p->off_off = off;
  off += align256((size_t)(nq + 1) * 4);
  p->off_temp = off;
  off += align256(p->temp_bytes);
  p->off_merge = off;
  off += align256(p->merge_bytes);
  p->off_codes = off;
  off += align256((size_t)nq * p->pmax * 8);
  p->off_scores = off;
  off += align256((size_t)nq * p->pmax * 4);
  p->total = off;
  return FX_OK;
}

}  // namespace

}  // namespace fx

using namespace fx;

extern "C" {

int fx_row_sqnorms(const void* x, int dtype, int64_t n, int64_t d, float* out, void* stream_) {
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
  if (n < 0 || d <= 0 || (n > 0 && (x == nullptr || out == nullptr))) {
    set_error("fx_row_sqnorms: invalid arguments");
    return FX_EINVAL;
  }
  if (dtype != FX_DTYPE_F32 && dtype != FX_DTYPE_F16) {
    set_error("unsupported dtype %d", dtype);
    return FX_EINVAL;
  }
  if (n == 0) return FX_OK;
  const dim3 grid((unsigned)((n + 3) / 4));
  if (dtype == FX_DTYPE_F32)
    hipLaunchKernelGGL(rownorm_kernel<float>, grid, dim3(256), 0, stream,
                       reinterpret_cast<const float*>(x), n, (int)d, 0, out);
  else
    hipLaunchKernelGGL(rownorm_kernel<_Float16>, grid, dim3(256), 0, stream,
                       reinterpret_cast<const _Float16*>(x), n, (int)d, 0, out);
  return check_launch("rownorm_kernel");
}

int fx_code_assign_workspace_bytes(int64_t n, int64_t d, int64_t nb, int64_t ks, size_t* out) {
  if (out == nullptr || n < 0 || d <= 0 || nb <= 0 || ks <= 0) {
    set_error("fx_code_assign_workspace_bytes: invalid arguments");
    return FX_EINVAL;
  }
  *out = assign_layout(1, n, nb, ks, d).total;
  return FX_OK;
}

int fx_code_assign(const void* x, int dtype, int64_t n, int64_t d, const float* codewords,
                   int64_t nb, int64_t ks, int metric, void* ws, size_t ws_bytes,
                   int32_t* out_index, int64_t* out_code, float* out_dist, void* stream_) {
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
  int rc = validate_code(n, d, dtype, nb, ks, metric);
  if (rc) return rc;
  if (composite_count(nb, ks) < 0 && out_code != nullptr) {
    set_error("composite code %lld^%lld does not fit 31 bits", (long long)ks, (long long)nb);
    return FX_EUNSUPPORTED;
  }
  const AssignLayout l = assign_layout(1, n, nb, ks, d);
  if (ws == nullptr || ws_bytes < l.total) {
    set_error("workspace too small: %zu < %zu", ws_bytes, l.total);
    return FX_EINVAL;
  }
  if (n == 0) return FX_OK;
  char* w = reinterpret_cast<char*>(ws);
  rc = run_assign(x, dtype, 1, n, d, codewords, nb, ks, metric, w, l, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(finalize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     reinterpret_cast<const uint64_t*>(w + l.off_keys), n, (int)nb, (int)ks,
                     metric, out_index, out_code, out_dist);
  return check_launch("finalize_kernel");
}

int fx_kmeans_step_workspace_bytes(int64_t nb, int64_t bs, int64_t d, int64_t ks, size_t* out) {
  if (out == nullptr || nb <= 0 || bs <= 0 || d <= 0 || ks <= 0) {
    set_error("fx_kmeans_step_workspace_bytes: invalid arguments");
    return FX_EINVAL;
  }
  const AssignLayout l = assign_layout(nb, bs, 1, ks, d);
  *out = l.total + align256((size_t)nb * bs * 4) * 2;
  return FX_OK;
}

int fx_kmeans_step(const void* sample, int dtype, int64_t nb, int64_t bs, int64_t d,
                   float* codewords, int64_t ks, int metric, void* ws, size_t ws_bytes,
                   void* stream_) {
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
  int rc = validate_code(nb * bs, d, dtype, nb, ks, metric);
  if (rc) return rc;
  if (bs <= 0 || sample == nullptr || codewords == nullptr) {
    set_error("fx_kmeans_step: invalid arguments");
    return FX_EINVAL;
  }
  if (d > kUpdDims * kUpdThreads) {
    set_error("fx_kmeans_step: d=%lld exceeds %d", (long long)d, kUpdDims * kUpdThreads);
    return FX_EUNSUPPORTED;
  }
  const AssignLayout l = assign_layout(nb, bs, 1, ks, d);
  const size_t need = l.total + align256((size_t)nb * bs * 4) * 2;
  if (ws == nullptr || ws_bytes < need) {
    set_error("workspace too small: %zu < %zu", ws_bytes, need);
    return FX_EINVAL;
  }
  char* w = reinterpret_cast<char*>(ws);
  int32_t* assign = reinterpret_cast<int32_t*>(w + l.total);
  float* rnorm = reinterpret_cast<float*>(w + l.total + align256((size_t)nb * bs * 4));
  const bool cosine = metric == FX_METRIC_COS;
  if (cosine) {  // update() normalises the codewords and the sample first (coder.py:54-56)
    const int64_t rows = nb * ks;
    hipLaunchKernelGGL(normalize_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream,
                       codewords, rows, (int)d);
    rc = check_launch("normalize_kernel");
    if (rc) return rc;
    const dim3 grid((unsigned)((nb * bs + 3) / 4));
    if (dtype == FX_DTYPE_F32)
      hipLaunchKernelGGL(rownorm_kernel<float>, grid, dim3(256), 0, stream,
                         reinterpret_cast<const float*>(sample), nb * bs, (int)d, 1, rnorm);
    else
      hipLaunchKernelGGL(rownorm_kernel<_Float16>, grid, dim3(256), 0, stream,
                         reinterpret_cast<const _Float16*>(sample), nb * bs, (int)d, 1, rnorm);
    rc = check_launch("rownorm_kernel");
    if (rc) return rc;
  }
  // argmin over each codebook for its own sample slice (vmap over codebooks)
  rc = run_assign(sample, dtype, nb, bs, d, codewords, 1, ks, metric, w, l, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(finalize_kernel, dim3((unsigned)((nb * bs + 255) / 256)), dim3(256), 0,
                     stream, reinterpret_cast<const uint64_t*>(w + l.off_keys), nb * bs, 1,
                     (int)ks, metric, assign, (int64_t*)nullptr, (float*)nullptr);
  rc = check_launch("finalize_kernel");
  if (rc) return rc;
  const dim3 grid((unsigned)ks, (unsigned)nb);
  if (dtype == FX_DTYPE_F32)
    hipLaunchKernelGGL(update_kernel<float>, grid, dim3(kUpdThreads), 0, stream,
                       reinterpret_cast<const float*>(sample), bs, (int)d, assign,
                       cosine ? rnorm : nullptr, codewords, (int)ks, cosine ? 1 : 0);
  else
    hipLaunchKernelGGL(update_kernel<_Float16>, grid, dim3(kUpdThreads), 0, stream,
                       reinterpret_cast<const _Float16*>(sample), bs, (int)d, assign,
                       cosine ? rnorm : nullptr, codewords, (int)ks, cosine ? 1 : 0);
  return check_launch("update_kernel");
}

int fx_code_probe_workspace_bytes(int64_t nq, int64_t nb, int64_t ks, size_t* out) {
  if (out == nullptr || nq <= 0 || nb <= 0 || ks <= 0) {
    set_error("fx_code_probe_workspace_bytes: invalid arguments");
    return FX_EINVAL;
  }
  ProbeLayout p;
  int rc = probe_layout(nq, nb, ks, &p);
  if (rc) return rc;
  *out = p.total;
  return FX_OK;
}

int fx_code_probe(const float* cw_dist, int64_t nq, int64_t nb, int64_t ks, int64_t probes,
                  void* ws, size_t ws_bytes, int64_t* out_code, float* out_score,
                  uint32_t* out_sel, void* stream_) {
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
  if (cw_dist == nullptr || nq <= 0 || nb <= 0 || ks <= 0) {
    set_error("fx_code_probe: invalid arguments");
    return FX_EINVAL;
  }
  ProbeLayout p;
  int rc = probe_layout(nq, nb, ks, &p);
  if (rc) return rc;
  if (probes <= 0 || probes > p.C) {
    set_error("probes %lld out of range for %lld composite codes", (long long)probes,
              (long long)p.C);
    return FX_EINVAL;
  }
  if (ws == nullptr || ws_bytes < p.total) {
    set_error("workspace too small: %zu < %zu", ws_bytes, p.total);
    return FX_EINVAL;
  }
  char* w = reinterpret_cast<char*>(ws);
  uint64_t* keys = reinterpret_cast<uint64_t*>(w + p.off_keys);
  const int64_t words = (p.C + 31) / 32;
  hipError_t e;
  if (out_sel != nullptr) {
    e = hipMemsetAsync(out_sel, 0, (size_t)nq * words * 4, stream);
    if (e != hipSuccess) {
      set_error("probe memset: %s", hipGetErrorString(e));
      return FX_EHIP;
    }
  }
  if (probes <= kProbeMerge) {
    hipLaunchKernelGGL(composite_lists_kernel,
                       dim3((unsigned)((p.padded + 255) / 256), (unsigned)nq), dim3(256), 0,
                       stream, cw_dist, (int)nb, (int)ks, p.C, p.padded, keys);
    rc = check_launch("composite_lists_kernel");
    if (rc) return rc;
    MergePlan mp;
    rc = plan_merge(nq, p.nlists, p.kin, probes, &mp);
    if (rc) return rc;
    if (mp.ws_bytes > p.merge_bytes) {
      set_error("probe merge workspace %zu > %zu", mp.ws_bytes, p.merge_bytes);
      return FX_EUNSUPPORTED;
    }
    int64_t* codes = out_code ? out_code : reinterpret_cast<int64_t*>(w + p.off_codes);
    float* scores = out_score ? out_score : reinterpret_cast<float*>(w + p.off_scores);
    rc = run_merge(mp, keys, nq, probes, w + p.off_merge, scores, codes, stream);
    if (rc) return rc;
    if (out_sel == nullptr) return FX_OK;
    hipLaunchKernelGGL(sel_kernel, dim3((unsigned)((probes + 255) / 256), (unsigned)nq),
                       dim3(256), 0, stream, codes, probes, out_sel, words);
    return check_launch("sel_kernel");
  }
  uint64_t* sorted = reinterpret_cast<uint64_t*>(w + p.off_sorted);
  int* off = reinterpret_cast<int*>(w + p.off_off);
  hipLaunchKernelGGL(composite_lists_kernel, dim3((unsigned)((p.C + 255) / 256), (unsigned)nq),
                     dim3(256), 0, stream, cw_dist, (int)nb, (int)ks, p.C, p.C, keys);
  rc = check_launch("composite_lists_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(offsets_kernel, dim3((unsigned)((nq + 256) / 256)), dim3(256), 0, stream, off,
                     nq, p.C);
  rc = check_launch("offsets_kernel");
  if (rc) return rc;
  size_t temp = p.temp_bytes;
  e = hipcub::DeviceSegmentedRadixSort::SortKeys(w + p.off_temp, temp, keys, sorted,
                                                 (int)(nq * p.C), (int)nq, off, off + 1, 0, 64,
                                                 stream);
  if (e != hipSuccess) {
    set_error("segmented sort: %s", hipGetErrorString(e));
    return FX_EHIP;
  }
  hipLaunchKernelGGL(emit_kernel, dim3((unsigned)((probes + 255) / 256), (unsigned)nq), dim3(256),
                     0, stream, sorted, p.C, probes, out_code, out_score, out_sel, words);
  return check_launch("emit_kernel");
}

int fx_code_mask(const int64_t* row_code, int64_t n, const uint32_t* sel, int64_t ncodes,
                 const uint32_t* filter, uint32_t* out_mask, uint64_t* out_count,
                 void* stream_) {
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
  if (n < 0 || ncodes <= 0 || (n > 0 && (row_code == nullptr || sel == nullptr ||
                                         out_mask == nullptr))) {
    set_error("fx_code_mask: invalid arguments");
    return FX_EINVAL;
  }
  if (out_count != nullptr) {
    hipError_t e = hipMemsetAsync(out_count, 0, 8, stream);
    if (e != hipSuccess) {
      set_error("mask memset: %s", hipGetErrorString(e));
      return FX_EHIP;
    }
  }
  if (n == 0) return FX_OK;
  const int64_t words = (n + 31) / 32;
  int cus = 0;
  int rc = device_cus(&cus);
  if (rc) return rc;
  int64_t blocks = (n + 255) / 256;
  if (blocks > (int64_t)cus * 8) blocks = (int64_t)cus * 8;
  hipLaunchKernelGGL(mask_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                     row_code, n, sel, ncodes, filter, out_mask, words,
                     reinterpret_cast<unsigned long long*>(out_count));
  return check_launch("mask_kernel");
}

}  // extern "C"

extern "C" {

int fx_mask_compact_workspace_bytes(int64_t n, size_t* out_bytes) {
  if (out_bytes == nullptr || n < 0) {
    set_error("fx_mask_compact_workspace_bytes: invalid arguments");
    return FX_EINVAL;
  }
  const int64_t words = (n + 31) / 32;
  const int64_t blocks = (words + kCompactWords - 1) / kCompactWords;
  *out_bytes = align256((size_t)(blocks > 0 ? blocks : 1) * 4);
  return FX_OK;
}

int fx_mask_compact(const uint32_t* mask, int64_t n, void* ws, size_t ws_bytes, int32_t* out_rows,
                    uint64_t* out_count, void* stream_) {
  hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
  if (n < 0 || n > 0x7fffffffll || (n > 0 && (mask == nullptr || out_rows == nullptr ||
                                               ws == nullptr))) {
    set_error("fx_mask_compact: invalid arguments");
    return FX_EINVAL;
  }
  const int64_t words = (n + 31) / 32;
  const int64_t blocks = (words + kCompactWords - 1) / kCompactWords;
  if (ws_bytes < (size_t)blocks * 4) {
    set_error("workspace too small: %zu < %zu", ws_bytes, (size_t)blocks * 4);
    return FX_EINVAL;
  }
  if (n == 0) {
    if (out_count == nullptr) return FX_OK;
    hipError_t e = hipMemsetAsync(out_count, 0, 8, stream);
    if (e != hipSuccess) {
      set_error("compact memset: %s", hipGetErrorString(e));
      return FX_EHIP;
    }
    return FX_OK;
  }
  uint32_t* counts = reinterpret_cast<uint32_t*>(ws);
  hipLaunchKernelGGL(compact_count_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, mask,
                     words, counts);
  int rc = check_launch("compact_count_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, stream, counts, blocks,
                     reinterpret_cast<unsigned long long*>(out_count));
  rc = check_launch("compact_scan_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(compact_write_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, mask,
                     words, counts, out_rows);
  return check_launch("compact_write_kernel");
}

}  // extern "C"
