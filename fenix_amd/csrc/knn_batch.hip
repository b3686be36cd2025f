// Batched-query search: fp32 MFMA GEMM with a fused threshold filter.
//
// The configs[2] workload (10M x 768 f32 cosine, 256 queries) is a true dense
// GEMM, S = X . Q^T, at 128 flop/byte — compute-bound on the matrix cores
// (SURVEY §8(d)).  The reference evaluates it as 256 separate searches of the
// per-chunk UDF (src/fenix/io/index/index.py:137-162 ->
// src/fenix/io/coder/coder.py:42-48); here one pass over the corpus serves
// every query.
//
// MFMA: v_mfma_f32_32x32x2_f32 (f32 in, f32 accumulate; bit-for-bit a K-ordered
// fmaf chain, cdna_hip_programming.md §3), so batched distances carry f32
// precision like the single-query scan.  Block = 4 waves (one per SIMD) =
// 128 rows x 256 queries; per 32-deep K chunk the block stages X[128][32] and
// Q[256][32] in LDS (rows padded to 36 floats: conflict-free ds_read_b128) and
// each wave issues 8 query tiles x 16 MFMAs.  The K order inside a chunk is
// permuted identically for A and B (lane half h reads k = 8g+4h..+3 with one
// ds_read_b128 and feeds element t to MFMA t).  Global->LDS staging for chunk
// c+1 is issued before chunk c's MFMAs (register prefetch, double-buffered LDS).
//
// Top-k without per-query lists in LDS (256 queries x k do not fit): the kernel
// appends every (row, query) whose composite is <= the query's threshold to a
// per-query candidate buffer in HBM (one atomic per append).  Thresholds come
// from earlier launches of the same kernel over row samples: the k-th
// composite of ANY subset of rows upper-bounds the global k-th, so filtering
// with it never drops a true top-k row (capi.hip: batched_search).  The
// buffers are then reduced by the ordinary merge kernels.
#include "fx_internal.h"
#include "fx_select.h"
#include "fx_wave.h"

namespace fx {

// The fp32-MFMA batch kernel was replaced by the fp16-MFMA filter
// (knn_filter.hip, 4-7x faster); it stays in diagnostic builds (tools/).
// The query norms and the exact rescoring below serve the filter.
#ifdef FX_DIAG_BUILD
#ifndef FX_BATCH_BQ
#define FX_BATCH_BQ 256  // queries per block: 256 (110 KB LDS, 1 block/CU) or 128 (74 KB, 2)
#endif
constexpr int kBM = 128;        // rows per block tile
constexpr int kBQ = FX_BATCH_BQ;  // queries per block
#ifndef FX_BATCH_BK
#define FX_BATCH_BK 32
#endif
#ifndef FX_BATCH_BPC
#define FX_BATCH_BPC (FX_BATCH_BQ == 256 ? 1 : 2)  // blocks per CU the LDS allows
#endif
constexpr int kBK = FX_BATCH_BK;  // K chunk
constexpr int kLds = kBK + 4;   // padded LDS row (floats)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct BatchShared {
  float xs[2][kBM * kLds];
  float qs[2][kBQ * kLds];
  float rownorm[kBM];
};

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

#ifndef FX_BATCH_WAVES
#define FX_BATCH_WAVES 8  // 4: one wave per SIMD; 8: two (4 row groups x 2 query halves)
#endif
constexpr int kWaves = FX_BATCH_WAVES;
constexpr int kThreads = 64 * kWaves;
constexpr int kQTiles = (kBQ / 32) * 4 / kWaves;  // 32-query MFMA tiles per wave
constexpr int kBlocksPerCU = FX_BATCH_BPC;
constexpr int kC4 = kBK / 4;  // 16-B pieces per row per chunk

// Stage one K chunk (columns [k0, k0+32)) of X rows [r0, r0+128) and of the
// query tile into registers (16-B pieces; 1024 of X, 2048 of Q per chunk).
struct Prefetch {
  f32x4 x[kBM * kC4 / kThreads];
  f32x4 q[kBQ * kC4 / kThreads];
};

__device__ __forceinline__ void prefetch_chunk(Prefetch& p, const BatchArgs& a, int64_t r0,
                                               int64_t q0, int k0, int tid) {
#pragma unroll
  for (int i = 0; i < kBM * kC4 / kThreads; ++i) {
    const int idx = i * kThreads + tid;  // row = idx/kC4, col4 = idx%kC4
    const int row = idx / kC4, c4 = idx % kC4;
    const int64_t gr = r0 + row;
    const int k = k0 + c4 * 4;
    if (gr < a.n && k < a.d) {
      p.x[i] = __builtin_nontemporal_load(
          reinterpret_cast<const f32x4*>(a.X + gr * (int64_t)a.d + k));
    } else {
      p.x[i] = f32x4(0.f);
    }
  }
#pragma unroll
  for (int i = 0; i < kBQ * kC4 / kThreads; ++i) {
    const int idx = i * kThreads + tid;  // query = idx/kC4, col4 = idx%kC4
    const int qq = idx / kC4, c4 = idx % kC4;
    const int64_t gq = q0 + qq;
    const int k = k0 + c4 * 4;
    p.q[i] = (gq < a.nq && k < a.d) ? ld4(a.Q + gq * (int64_t)a.d + k) : f32x4(0.f);
  }
}

__device__ __forceinline__ void store_chunk(const Prefetch& p, BatchShared* sh, int buf, int tid) {
#pragma unroll
  for (int i = 0; i < kBM * kC4 / kThreads; ++i) {
    const int idx = i * kThreads + tid;
    *reinterpret_cast<f32x4*>(&sh->xs[buf][(idx / kC4) * kLds + (idx % kC4) * 4]) = p.x[i];
  }
#pragma unroll
  for (int i = 0; i < kBQ * kC4 / kThreads; ++i) {
    const int idx = i * kThreads + tid;
    *reinterpret_cast<f32x4*>(&sh->qs[buf][(idx / kC4) * kLds + (idx % kC4) * 4]) = p.q[i];
  }
}

template <int METRIC>
// second argument: minimum waves per SIMD (kWaves * blocks per CU / 4 SIMDs)
__global__ void __launch_bounds__(kThreads, kWaves * kBlocksPerCU / 4) batch_kernel(BatchArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  BatchShared* sh = reinterpret_cast<BatchShared*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int rg = wid & 3;                   // 32-row group of this wave
  const int qtile0 = (wid >> 2) * kQTiles;  // first 32-query tile of this wave
  const int h = lane >> 5, l32 = lane & 31;
  const int64_t q0 = (int64_t)blockIdx.y * kBQ;
  const int nchunks = (a.d + kBK - 1) / kBK;

  // per-lane query state for its query columns
  uint64_t thr[kQTiles];
  float qn[kQTiles];
#pragma unroll
  for (int qt = 0; qt < kQTiles; ++qt) {
    const int64_t gq = q0 + (qtile0 + qt) * 32 + l32;
    thr[qt] = gq < a.nq ? a.thr[gq] : 0ull;
    qn[qt] = gq < a.nq ? a.qnorm[gq] : 1.f;
  }

  for (int64_t ti = blockIdx.x; ti < a.num_tiles; ti += gridDim.x) {
    const int64_t tile = a.tile_start + ti * a.tile_stride;
    const int64_t r0 = tile * kBM;
    if (r0 >= a.n) continue;

    f32x16 acc[kQTiles];
#pragma unroll
    for (int qt = 0; qt < kQTiles; ++qt) acc[qt] = f32x16(0.f);
    float sumsq = 0.f;

    Prefetch pf;
    prefetch_chunk(pf, a, r0, q0, 0, tid);
    __syncthreads();  // previous tile's epilogue is done with the LDS
    store_chunk(pf, sh, 0, tid);
    __syncthreads();

    for (int c = 0; c < nchunks; ++c) {
      const int buf = c & 1;
      if (c + 1 < nchunks) prefetch_chunk(pf, a, r0, q0, (c + 1) * kBK, tid);
      const float* xs = sh->xs[buf] + (rg * 32 + l32) * kLds + 4 * h;
      const float* qs = sh->qs[buf] + (qtile0 * 32 + l32) * kLds + 4 * h;
#pragma unroll
      for (int g = 0; g < kBK / 8; ++g) {
        const f32x4 av = ld4(xs + 8 * g);
        if constexpr (METRIC != 1) {
          sumsq = fmaf(av[0], av[0], sumsq);
          sumsq = fmaf(av[1], av[1], sumsq);
          sumsq = fmaf(av[2], av[2], sumsq);
          sumsq = fmaf(av[3], av[3], sumsq);
        }
#pragma unroll
        for (int qt = 0; qt < kQTiles; ++qt) {
          const f32x4 bv = ld4(qs + qt * 32 * kLds + 8 * g);
#pragma unroll
          for (int t = 0; t < 4; ++t)
            acc[qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[t], bv[t], acc[qt], 0, 0, 0);
        }
      }
      if (c + 1 < nchunks) store_chunk(pf, sh, buf ^ 1, tid);
      __syncthreads();
    }

    // ---- epilogue: distances, threshold filter, append
    if constexpr (METRIC == 2) {
      sumsq += __shfl_xor(sumsq, 32);
      if (h == 0 && qtile0 == 0) sh->rownorm[rg * 32 + l32] = fmaxf(sqrtf(sumsq), 1e-12f);
    } else if constexpr (METRIC == 0) {
      sumsq += __shfl_xor(sumsq, 32);
      if (h == 0 && qtile0 == 0) sh->rownorm[rg * 32 + l32] = sumsq;  // |x|^2
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int lr = rg * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int64_t row = r0 + lr;
      bool ok = row < a.n;
      if (ok && a.mask != nullptr) ok = (a.mask[row >> 5] >> (row & 31)) & 1u;
      float nx = 1.f;
      if constexpr (METRIC != 1) nx = sh->rownorm[lr];
#pragma unroll
      for (int qt = 0; qt < kQTiles; ++qt) {
        const float dot = acc[qt][r];
        float dist;
        bool pass;
        uint64_t comp;
        if constexpr (METRIC == 0) {
          // |x-q|^2 by expansion: an approximation whose fp32 error is at most
          // l2_eps * (|x|^2 + |q|^2); a row passes if its lower bound can be
          // within the threshold, and is rescored exactly (rescore_kernel)
          // before any threshold or result is taken from it.
          const float s2 = nx + qn[qt];
          const float d2 = fmaxf(s2 - 2.f * dot, 0.f);
          const float lo = fmaxf(d2 - a.l2_eps * s2, 0.f);
          comp = make_comp(d2, (uint32_t)(a.row_base + row));
          pass = order_key(sqrtf(lo)) <= (uint32_t)(thr[qt] >> 32);
        } else {
          if constexpr (METRIC == 1) {
            dist = -dot;
          } else {
            dist = 0.5f - 0.5f * (dot / (nx * qn[qt]));
          }
          comp = make_comp(dist, (uint32_t)(a.row_base + row));
          pass = comp <= thr[qt];
        }
        if (ok && pass) {
          const int64_t gq = q0 + (qtile0 + qt) * 32 + l32;
          const uint32_t pos = atomicAdd(&a.count[gq * kCountStride], 1u);
          if (pos < (uint32_t)a.cap) a.cand[gq * a.cap + pos] = comp;
        }
      }
    }
  }
}

int launch_batch(const BatchArgs& a, int metric, hipStream_t stream) {
  if (a.num_tiles <= 0) return FX_OK;
  const size_t smem = sizeof(BatchShared);
  const void* fn = metric == FX_METRIC_COS ? (const void*)batch_kernel<2>
                   : metric == FX_METRIC_IP ? (const void*)batch_kernel<1>
                                            : (const void*)batch_kernel<0>;
  if (int rc = allow_lds(fn)) return rc;
  int cus = 0;
  int rc = device_cus(&cus);
  if (rc) return rc;
  const int64_t qtiles = (a.nq + kBQ - 1) / kBQ;
  int64_t bx = (int64_t)cus * kBlocksPerCU;
  if (bx > a.num_tiles) bx = a.num_tiles;
  for (int64_t y0 = 0; y0 < qtiles; y0 += 65535) {
    BatchArgs b = a;
    const int64_t yn = (qtiles - y0) < 65535 ? (qtiles - y0) : 65535;
    b.Q = a.Q + y0 * kBQ * (int64_t)a.d;
    b.qnorm = a.qnorm + y0 * kBQ;
    b.thr = a.thr + y0 * kBQ;
    b.count = a.count + y0 * kBQ * kCountStride;
    b.cand = a.cand + y0 * kBQ * (int64_t)a.cap;
    b.nq = a.nq - y0 * kBQ;
    void* args[] = {(void*)&b};
    hipError_t e = hipLaunchKernel(fn, dim3((unsigned)bx, (unsigned)yn), dim3(kThreads), args, smem,
                                   stream);
    if (e != hipSuccess) {
      set_error("batch_kernel launch: %s", hipGetErrorString(e));
      return FX_EHIP;
    }
  }
  return check_launch("batch_kernel");
}

#endif  // FX_DIAG_BUILD

int batch_tile_rows() { return 128; }

// cosine: max(||q||, 1e-12) per query (F.normalize eps, coder.py:43-44);
// L2 (mode 1): sum of squares for the expansion
__global__ void qnorm_kernel(const float* __restrict__ Q, int64_t nq, int d, float* __restrict__ out,
                             int mode) {
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (q >= nq) return;
  float s = 0.f;
  for (int i = lane; i < d; i += 64) s = fmaf(Q[q * d + i], Q[q * d + i], s);
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  if (lane == 0) out[q] = mode == 1 ? s : fmaxf(sqrtf(s), 1e-12f);
}

int launch_qnorm(const float* Q, int64_t nq, int d, float* out, hipStream_t stream, int mode) {
  hipLaunchKernelGGL(qnorm_kernel, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, stream, Q, nq, d,
                     out, mode);
  return check_launch("qnorm_kernel");
}

// The single-query scan's f32 distance of one row, computed by a 16-lane
// group (lane jl of the group): 16-B loads of the row and the query, the
// scan's per-lane fmaf chain over slots jl, jl+16, ... (knn_scan.hip
// tile_accumulate), its sum16 reduction and its distance formula
// (tile_finish): bit for bit the scan's value.  Every lane of the wave must
// call it (sum16 is a cross-lane reduction); live = false contributes zeros.
template <typename T, int METRIC>
__device__ __forceinline__ float exact_distance16(const T* __restrict__ xr,
                                                  const float* __restrict__ qv, int d, int jl,
                                                  bool live, float qnorm) {
  // the scan's 16-B slots: 4 floats (f32) or 8 halves (f16), lane jl takes
  // slots jl, jl + 16, ... (knn_scan.hip plan_scan: W = 16 / sizeof(T))
  constexpr int W = 16 / sizeof(T);
  constexpr int S = 16 * W;  // elements between a lane's slots
  typedef T vT __attribute__((ext_vector_type(W)));
  typedef float vF __attribute__((ext_vector_type(W)));
  float acc = 0.f, acc2 = 0.f;
  auto slot = [&](const vT& xv, const vF& yv) {
#pragma unroll
    for (int t = 0; t < W; ++t) {
      const float x = (float)xv[t];
      const float y = yv[t];
      if constexpr (METRIC == 0) {
        const float df = x - y;
        acc = fmaf(df, df, acc);
      } else if constexpr (METRIC == 1) {
        acc = fmaf(x, y, acc);
      } else {
        acc = fmaf(x, y, acc);
        acc2 = fmaf(x, x, acc2);
      }
    }
  };
  // NS slots of the lane loaded at once (all of a 768-d f32 or a 1024-d f16
  // row), then multiplied in the scan's order
  constexpr int NS = W == 4 ? 12 : 8;
  if (live) {
    for (int base = jl * W; base < d; base += NS * S) {
      vT xv[NS];
      vF yv[NS];
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        const int k = base + i * S;
        if (k < d) {
          xv[i] = *reinterpret_cast<const vT*>(xr + k);
          yv[i] = *reinterpret_cast<const vF*>(qv + k);
        }
      }
#pragma unroll
      for (int i = 0; i < NS; ++i)
        if (base + i * S < d) slot(xv[i], yv[i]);
    }
  }
  const float s1 = sum16(acc);  // the scan's reduction: bit-identical distances
  if constexpr (METRIC == 0) {
    return sqrtf(s1);
  } else if constexpr (METRIC == 1) {
    return -s1;
  } else {
    const float s2 = sum16(acc2);
    const float nx = fmaxf(sqrtf(s2), 1e-12f);
    return 0.5f - 0.5f * (s1 / (nx * qnorm));
  }
}

// Exact distance of each appended candidate (exact_distance16); the key is
// replaced in place (row unchanged).  With thr, a candidate whose
// (lower-bound) key is above the query's threshold key is dropped (kEmpty)
// unread.  Each wave takes 64 slots at a time, one per lane, and rescores the
// kept ones 4 at a time (a 16-lane group each, the kept lanes taken in order
// from the wave's ballot): dropped candidates cost one load and no group.
// Small query counts (kRescoreDenseMaxQ), whose candidates are mostly kept:
// every 16-lane group takes its own slot (4 per wave per step), so a few
// thousand candidates cost one round trip each across the whole grid
// instead of up to 16 rounds per wave (single query, 3.3 K candidates: ~25
// -> a few us).
constexpr unsigned kRescoreDenseMaxQ = 2;
template <typename T, int METRIC>
__global__ void __launch_bounds__(256) rescore_dense_kernel(const T* __restrict__ X, int64_t n,
                                                            int d, int64_t row_base,
                                                            const float* __restrict__ Q,
                                                            const float* __restrict__ qnorm,
                                                            const uint32_t* __restrict__ count,
                                                            uint64_t* __restrict__ cand, int cap,
                                                            const uint64_t* __restrict__ thr) {
  const int64_t q = blockIdx.y;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int grp = lane >> 4, jl = lane & 15;
  const uint32_t cq = count[q * kCountStride];
  const int64_t cnt = cq < (uint32_t)cap ? cq : (uint32_t)cap;
  const uint32_t tkey = thr != nullptr ? (uint32_t)(thr[q] >> 32) : 0xffffffffu;
  const float* qv = Q + q * (int64_t)d;
  const float qn = METRIC == 2 ? qnorm[q] : 0.f;
  uint64_t* cl = cand + q * (int64_t)cap;
  for (int64_t base = ((int64_t)blockIdx.x * 4 + wv) * 4; base < cnt;
       base += (int64_t)gridDim.x * 16) {  // wave-uniform trip count
    const int64_t i = base + grp;
    const uint64_t c = i < cnt ? cl[i] : kEmpty;
    const int64_t row = (int64_t)(c & 0xffffffffull) - row_base;
    const bool keep = c != kEmpty && (uint32_t)(c >> 32) <= tkey && row >= 0 && row < n;
    const float dist =
        exact_distance16<T, METRIC>(X + (keep ? row : 0) * (int64_t)d, qv, d, jl, keep, qn);
    if (jl == 0 && c != kEmpty)
      cl[i] = keep ? make_comp(dist, (uint32_t)(c & 0xffffffffull)) : kEmpty;
  }
}

template <typename T, int METRIC>
__global__ void __launch_bounds__(256) rescore_kernel(const T* __restrict__ X, int64_t n, int d,
                                                      int64_t row_base,
                                                      const float* __restrict__ Q,
                                                      const float* __restrict__ qnorm,
                                                      const uint32_t* __restrict__ count,
                                                      uint64_t* __restrict__ cand, int cap,
                                                      const uint64_t* __restrict__ thr) {
  const int64_t q = blockIdx.y;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int grp = lane >> 4, jl = lane & 15;
  const uint32_t cq = count[q * kCountStride];
  const int64_t cnt = cq < (uint32_t)cap ? cq : (uint32_t)cap;
  const uint32_t tkey = thr != nullptr ? (uint32_t)(thr[q] >> 32) : 0xffffffffu;
  const float* qv = Q + q * (int64_t)d;
  const float qn = METRIC == 2 ? qnorm[q] : 0.f;
  uint64_t* cl = cand + q * (int64_t)cap;
  for (int64_t base = ((int64_t)blockIdx.x * 4 + wv) * 64; base < cnt;
       base += (int64_t)gridDim.x * 256) {  // wave-uniform trip count
    const int64_t i = base + lane;
    const uint64_t c = i < cnt ? cl[i] : kEmpty;
    const int64_t row = (int64_t)(c & 0xffffffffull) - row_base;
    const bool keep = c != kEmpty && (uint32_t)(c >> 32) <= tkey && row >= 0 && row < n;
    if (c != kEmpty && !keep) cl[i] = kEmpty;
    uint64_t m = __ballot(keep);
    while (m != 0ull) {  // wave-uniform: groups 0..3 take the next 4 kept lanes
      int src = -1;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int l = m != 0ull ? __builtin_ctzll(m) : -1;
        if (m != 0ull) m &= m - 1ull;
        if (g == grp) src = l;
      }
      const int from = src >= 0 ? src : 0;
      const uint32_t lo = __shfl((uint32_t)c, from), hi = __shfl((uint32_t)(c >> 32), from);
      const uint64_t cs = ((uint64_t)hi << 32) | lo;
      const int64_t rs = (int64_t)lo - row_base;
      const bool live = src >= 0;
      const float dist =
          exact_distance16<T, METRIC>(X + (live ? rs : 0) * (int64_t)d, qv, d, jl, live, qn);
      if (jl == 0 && live) cl[base + src] = make_comp(dist, (uint32_t)(cs & 0xffffffffull));
    }
  }
}

// Exact threshold from a query's k best candidates by upper bound (rows
// [nq][k], run_merge's out_row, -1 = missing): their exact distances
// (exact_distance16) are k rows' scan distances, so the largest composite
// bounds the k-th smallest from above; thr[q] = min(thr[q], it).  Two
// launches: exact_kth_kernel replaces each row in place by its exact
// composite (a missing row by the largest composite, so a query with fewer
// than k candidates keeps its threshold), grid (ceil(k / 16), nq), one row
// per 16-lane group; kth_max_kernel folds a query's k composites, one wave
// per query.  (One launch with a per-query block ticket behind a
// __threadfence took ~100 us for 256 x 100 rows: the blocks' fences and
// returning atomics, not the row loads, set its time.)
template <typename T, int METRIC>
__global__ void __launch_bounds__(256) exact_kth_kernel(const T* __restrict__ X, int64_t n, int d,
                                                        int64_t row_base,
                                                        const float* __restrict__ Q,
                                                        const float* __restrict__ qnorm, int k,
                                                        int64_t* __restrict__ rows) {
  const int64_t q = blockIdx.y;
  const int grp = threadIdx.x >> 4, jl = threadIdx.x & 15;
  const int j = blockIdx.x * 16 + grp;
  const int64_t grow = j < k ? rows[q * (int64_t)k + j] : 0;
  const int64_t row = grow - row_base;
  const bool live = j < k && grow >= 0 && row >= 0 && row < n;
  const float qn = METRIC == 2 ? qnorm[q] : 0.f;
  const float dist = exact_distance16<T, METRIC>(X + (live ? row : 0) * (int64_t)d,
                                                 Q + q * (int64_t)d, d, jl, live, qn);
  if (jl == 0 && j < k)
    rows[q * (int64_t)k + j] = live ? (int64_t)make_comp(dist, (uint32_t)grow) : (int64_t)kEmpty;
}

__global__ void __launch_bounds__(256) kth_max_kernel(const uint64_t* __restrict__ comps,
                                                      int64_t nq, int k,
                                                      uint64_t* __restrict__ thr) {
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (q >= nq) return;
  uint64_t m = 0ull;
  for (int j = lane; j < k; j += 64) {
    const uint64_t c = comps[q * (int64_t)k + j];
    m = c > m ? c : m;
  }
  m = wave_max_u64(m);
  if (lane == 0 && m < thr[q]) thr[q] = m;
}

template <typename T>
static void launch_rescore_t(const T* X, int64_t n, int d, int64_t row_base, const float* Q,
                             const float* qnm, const uint32_t* count, uint64_t* cand, int cap,
                             int metric, const uint64_t* t, dim3 grid, hipStream_t stream) {
  if (grid.y <= kRescoreDenseMaxQ) {
    // (one slot per 16-lane group: 16 K slots per grid step, fewer blocks
    // when the buffer is smaller)
    dim3 g2 = grid;
    const int64_t need = ((int64_t)cap + 15) / 16;
    g2.x = (unsigned)(need < 1024 ? need : 1024);
    if (metric == FX_METRIC_COS)
      hipLaunchKernelGGL((rescore_dense_kernel<T, 2>), g2, dim3(256), 0, stream, X, n, d,
                         row_base, Q, qnm, count, cand, cap, t);
    else if (metric == FX_METRIC_IP)
      hipLaunchKernelGGL((rescore_dense_kernel<T, 1>), g2, dim3(256), 0, stream, X, n, d,
                         row_base, Q, qnm, count, cand, cap, t);
    else
      hipLaunchKernelGGL((rescore_dense_kernel<T, 0>), g2, dim3(256), 0, stream, X, n, d,
                         row_base, Q, qnm, count, cand, cap, t);
    return;
  }
  if (metric == FX_METRIC_COS) {
    hipLaunchKernelGGL((rescore_kernel<T, 2>), grid, dim3(256), 0, stream, X, n, d, row_base, Q,
                       qnm, count, cand, cap, t);
  } else if (metric == FX_METRIC_IP) {
    hipLaunchKernelGGL((rescore_kernel<T, 1>), grid, dim3(256), 0, stream, X, n, d, row_base, Q,
                       qnm, count, cand, cap, t);
  } else {
    hipLaunchKernelGGL((rescore_kernel<T, 0>), grid, dim3(256), 0, stream, X, n, d, row_base, Q,
                       qnm, count, cand, cap, t);
  }
}

int launch_rescore(const void* X, int dtype, int64_t n, int d, int64_t row_base, const float* Q,
                   const float* qnorm, int64_t nq, const uint32_t* count, uint64_t* cand,
                   int cap, int metric, const uint64_t* thr, hipStream_t stream) {
  int cus = 0;
  int rc = device_cus(&cus);
  if (rc) return rc;
  // enough blocks for ~8 per CU over the batch, at most one per 256 slots
  int64_t bx = ((int64_t)cus * 8 + nq - 1) / (nq > 0 ? nq : 1);
  if (bx > ((int64_t)cap + 255) / 256) bx = ((int64_t)cap + 255) / 256;
  if (bx < 1) bx = 1;
  for (int64_t q0 = 0; q0 < nq; q0 += 65535) {
    const int64_t qn = (nq - q0) < 65535 ? (nq - q0) : 65535;
    const dim3 grid((unsigned)bx, (unsigned)qn);
    const uint64_t* t = thr != nullptr ? thr + q0 : nullptr;
    const float* qnm = qnorm != nullptr ? qnorm + q0 : nullptr;
    const uint32_t* cn = count + q0 * kCountStride;
    uint64_t* cd = cand + q0 * (int64_t)cap;
    if (dtype == FX_DTYPE_F16) {
      launch_rescore_t(reinterpret_cast<const _Float16*>(X), n, d, row_base, Q + q0 * d, qnm, cn,
                       cd, cap, metric, t, grid, stream);
    } else {
      launch_rescore_t(reinterpret_cast<const float*>(X), n, d, row_base, Q + q0 * d, qnm, cn, cd,
                       cap, metric, t, grid, stream);
    }
    rc = check_launch("rescore_kernel");
    if (rc) return rc;
  }
  return FX_OK;
}

template <typename T>
static void launch_exact_kth_t(const T* X, int64_t n, int d, int64_t row_base, const float* Q,
                               const float* qnm, int k, int64_t* rows, int metric, dim3 grid,
                               hipStream_t stream) {
  if (metric == FX_METRIC_COS) {
    hipLaunchKernelGGL((exact_kth_kernel<T, 2>), grid, dim3(256), 0, stream, X, n, d, row_base,
                       Q, qnm, k, rows);
  } else if (metric == FX_METRIC_IP) {
    hipLaunchKernelGGL((exact_kth_kernel<T, 1>), grid, dim3(256), 0, stream, X, n, d, row_base,
                       Q, qnm, k, rows);
  } else {
    hipLaunchKernelGGL((exact_kth_kernel<T, 0>), grid, dim3(256), 0, stream, X, n, d, row_base,
                       Q, qnm, k, rows);
  }
}

int launch_exact_kth(const void* X, int dtype, int64_t n, int d, int64_t row_base,
                     const float* Q, const float* qnorm, int64_t nq, int k, int64_t* rows,
                     int metric, uint64_t* thr, hipStream_t stream) {
  for (int64_t q0 = 0; q0 < nq; q0 += 65535) {
    const int64_t qn = (nq - q0) < 65535 ? (nq - q0) : 65535;
    const dim3 grid((unsigned)((k + 15) / 16), (unsigned)qn);
    const float* qnm = qnorm != nullptr ? qnorm + q0 : nullptr;
    if (dtype == FX_DTYPE_F16) {
      launch_exact_kth_t(reinterpret_cast<const _Float16*>(X), n, d, row_base, Q + q0 * d, qnm, k,
                         rows + q0 * k, metric, grid, stream);
    } else {
      launch_exact_kth_t(reinterpret_cast<const float*>(X), n, d, row_base, Q + q0 * d, qnm, k,
                         rows + q0 * k, metric, grid, stream);
    }
    int rc = check_launch("exact_kth_kernel");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(kth_max_kernel, dim3((unsigned)((nq + 3) / 4)), dim3(256), 0, stream,
                     reinterpret_cast<const uint64_t*>(rows), nq, k, thr);
  return check_launch("kth_max_kernel");
}

// One workgroup per query selects the k smallest keys among the query's
// first count[q] entries of keys [nq][cap] (a streaming block_keep_k over
// LDS-sized chunks, the k kept so far carried into the next chunk: any
// count in one launch), then
//   MODE 0 (exact threshold): their exact distances (exact_distance16, 64
//     groups of 16 lanes) and thr[q] = min(thr[q], the largest exact
//     composite) -- run_merge + launch_exact_kth in one launch; a query with
//     fewer than k candidates keeps its threshold;
//   MODE 1 (final select): the k smallest (exact composites after
//     launch_rescore) bitonic-sorted and decoded to (distance, row), the
//     last level of run_merge; a query whose count exceeds alt_gate (it
//     overflowed the buffer) selects from its alt_m entries of alt instead
//     (the overflow fallback scan's lists, [nq][alt_m]);
//   MODE 2 (sample threshold): thr[q] = min(thr[q], the k-th smallest key)
//     when there are at least k (run_merge's threshold-only level);
//   MODE 3 (prune, before a MODE 0/1/2 launch over many candidates): grid
//     (pre_p, nq), workgroup p keeps the k smallest of the query's entries
//     [p pre_s, (p + 1) pre_s) and writes them (kEmpty-padded) to
//     pre[q][p][k]; the MODE 0/1/2 launch given the same pre then selects
//     from the ceil(m / pre_s) k-lists of pre instead of streaming all m
//     entries through one workgroup (k = 1 000, ~100 K candidates: the
//     one-workgroup select took 160-230 us).  Not for the overflow path's
//     alt lists.
// zero_count resets the count once every thread has read it.
#ifndef FX_SELECT_THREADS
#define FX_SELECT_THREADS 1024
#endif
constexpr int kSelectThreads = FX_SELECT_THREADS;

// overflow_gate_kernel's arithmetic (knn_filter.hip, launch_overflow_gate) in
// the exact-threshold select's own workgroup, on the threshold it just set:
// the query's c appended lb composites of cand under thr, scaled by num / den
// and added to c; a query predicted past cap gets count = cap + 1.  Saves the
// gate's own launch (~5 us per search, profiles/r06_cfg1_img8_timeline.txt).
// Every thread calls it (barriers inside).
__device__ __forceinline__ void select_gate(const uint64_t* __restrict__ cand,
                                            uint32_t* __restrict__ count, int64_t q, uint32_t c,
                                            int64_t cap, uint64_t thrq, int64_t num, int64_t den,
                                            MergeShared* ms) {
  if (c > (uint32_t)cap) return;  // (uniform; already overflowing: recomputed anyway)
  const int tid = threadIdx.x;
  if (tid == 0) ms->ctr_eq = 0u;
  __syncthreads();
  const uint32_t t = (uint32_t)(thrq >> 32);
  const uint64_t* cq = cand + q * cap;
  uint32_t mine = 0u;
  for (uint32_t b = tid; b < c; b += kSelectThreads * 8) {
    uint64_t e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i = b + j * kSelectThreads;
      e[j] = i < c ? cq[i] : kEmpty;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) mine += b + j * kSelectThreads < c && (uint32_t)(e[j] >> 32) <= t;
  }
  for (int o = 32; o >= 1; o >>= 1) mine += __shfl_xor(mine, o);
  if ((tid & 63) == 0) atomicAdd(&ms->ctr_eq, mine);
  __syncthreads();
  if (tid == 0) {
    const uint64_t predicted =
        (uint64_t)c + ((uint64_t)ms->ctr_eq * (uint64_t)num + (uint64_t)den - 1) / (uint64_t)den;
    if (predicted > (uint64_t)cap) count[q * kCountStride] = (uint32_t)cap + 1u;
  }
}
constexpr int kSelectEntries = 16384;  // LDS chunk (128 KB)
template <typename T, int METRIC, int MODE>
__global__ void __launch_bounds__(kSelectThreads)
    select_kernel(const T* __restrict__ X, int64_t n, int d, int64_t row_base,
                  const float* __restrict__ Q, const float* __restrict__ qnorm,
                  const uint64_t* __restrict__ keys, int64_t cap, uint32_t* __restrict__ count,
                  int zero_count, int k, int P2, uint64_t* __restrict__ thr,
                  float* __restrict__ out_dist, int64_t* __restrict__ out_row,
                  const uint64_t* __restrict__ alt, int64_t alt_m, int64_t alt_gate,
                  uint64_t* __restrict__ pre, int pre_p, int64_t pre_s,
                  const uint64_t* __restrict__ gate_cand, int64_t gate_num, int64_t gate_den) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  MergeShared* ms = reinterpret_cast<MergeShared*>(smem);
  uint64_t* res = reinterpret_cast<uint64_t*>(smem + sizeof(MergeShared));
  uint64_t* s = res + P2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int64_t q = blockIdx.y;
  const uint32_t c = count[q * kCountStride];
  int64_t m = (int64_t)c < cap ? (int64_t)c : cap;
  const uint64_t* src = keys + q * cap;
  bool use_alt = false;
  if (MODE == 1 && alt != nullptr && (int64_t)c > alt_gate) {
    m = alt_m;
    src = alt + q * alt_m;
    use_alt = true;
  }
  if constexpr (MODE == 3) {
    const int64_t lo = (int64_t)blockIdx.x * pre_s;
    if (use_alt || lo >= m) return;  // (uniform)
    const int cnt = (int)((m - lo) < pre_s ? (m - lo) : pre_s);
    uint64_t* out = pre + (q * pre_p + blockIdx.x) * (int64_t)k;
    block_reset(ms);
    __syncthreads();
    uint64_t v_or = 0, v_and = ~0ull;
    for (int base = tid; base < cnt; base += kSelectThreads * 8) {
      uint64_t e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = base + j * kSelectThreads;
        e[j] = i < cnt ? src[lo + i] : kEmpty;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = base + j * kSelectThreads;
        if (i < cnt) {
          s[i] = e[j];
          v_or |= e[j];
          v_and &= e[j];
        }
      }
    }
    block_or_and(v_or, v_and, ms);
    __syncthreads();
    if (cnt > k) {
      block_keep_k<kSelectThreads>(s, cnt, k, out, ms);
    } else {
      for (int i = tid; i < k; i += kSelectThreads) out[i] = i < cnt ? s[i] : kEmpty;
    }
    return;
  }
  __syncthreads();
  if (zero_count && tid == 0) count[q * kCountStride] = 0u;
  if (MODE != 1 && m < k) {  // (uniform) fewer than k candidates: no threshold
    if (MODE == 0 && out_row != nullptr)  // (rows out: none, the query keeps its threshold)
      for (int i = tid; i < k; i += kSelectThreads) out_row[q * k + i] = -1;
    if (MODE == 0 && out_row == nullptr && gate_cand != nullptr)
      select_gate(gate_cand, count, q, c, cap, thr[q], gate_num, gate_den, ms);
    return;
  }
  if (pre != nullptr && !use_alt) {  // the pruned k-lists of the same entries (MODE 3)
    src = pre + q * pre_p * (int64_t)k;
    m = (m + pre_s - 1) / pre_s * k;
  }
  int nres = 0;
  const int64_t chunk = kSelectEntries - k;
  for (int64_t off = 0; off < m || (off == 0 && m == 0); off += chunk) {  // (uniform)
    const int cnt = (int)((m - off) < chunk ? (m - off) : chunk);
    block_reset(ms);
    __syncthreads();
    uint64_t v_or = 0, v_and = ~0ull;
    for (int base = tid; base < cnt; base += kSelectThreads * 8) {
      uint64_t e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = base + j * kSelectThreads;
        e[j] = i < cnt ? src[off + i] : kEmpty;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = base + j * kSelectThreads;
        if (i < cnt) {
          s[i] = e[j];
          v_or |= e[j];
          v_and &= e[j];
        }
      }
    }
    for (int i = tid; i < nres; i += kSelectThreads) {  // the k kept so far
      const uint64_t e = res[i];
      s[cnt + i] = e;
      v_or |= e;
      v_and &= e;
    }
    const int t = cnt + nres;
    block_or_and(v_or, v_and, ms);
    __syncthreads();
    if (t > k) {
      block_keep_k<kSelectThreads>(s, t, k, res, ms);
      nres = k;
    } else {
      for (int i = tid; i < t; i += kSelectThreads) res[i] = s[i];
      nres = t;
    }
    __syncthreads();
    if (m == 0) break;
  }
  if constexpr (MODE == 2) {
    uint64_t mx = 0ull;  // (nres == k: m >= k)
    for (int i = tid; i < nres; i += kSelectThreads) mx = res[i] > mx ? res[i] : mx;
    mx = wave_max_u64(mx);
    if (tid == 0) ms->shmax = 0ull;
    __syncthreads();
    if (lane == 0) atomicMax(&ms->shmax, (unsigned long long)mx);
    __syncthreads();
    if (tid == 0 && ms->shmax < thr[q]) thr[q] = ms->shmax;
  } else if constexpr (MODE == 0) {
    if (out_row != nullptr) {  // rows out: rescored by the whole chip (launch_exact_kth)
      for (int j = tid; j < k; j += kSelectThreads) {
        const uint64_t e = j < nres ? res[j] : kEmpty;
        out_row[q * k + j] = e == kEmpty ? -1 : (int64_t)(e & 0xffffffffull);
      }
      return;
    }
    if (tid == 0) ms->shmax = 0ull;
    __syncthreads();
    const int grp = tid >> 4, jl = tid & 15;
    const float* qv = Q + q * (int64_t)d;
    const float qn = METRIC == 2 ? qnorm[q] : 0.f;
    uint64_t mx = 0ull;
    for (int j0 = 0; j0 < k; j0 += kSelectThreads / 16) {  // (uniform trip count)
      const int j = j0 + grp;
      const uint64_t e = j < nres ? res[j] : kEmpty;
      const int64_t grow = (int64_t)(e & 0xffffffffull);
      const int64_t row = grow - row_base;
      const bool live = j < nres && e != kEmpty && row >= 0 && row < n;
      const float dist = exact_distance16<T, METRIC>(X + (live ? row : 0) * (int64_t)d, qv, d,
                                                     jl, live, qn);
      // a missing or out-of-shard row: the largest composite (no threshold)
      const uint64_t comp = live ? make_comp(dist, (uint32_t)grow) : kEmpty;
      if (j < k) mx = comp > mx ? comp : mx;
    }
    mx = wave_max_u64(mx);
    if (lane == 0) atomicMax(&ms->shmax, (unsigned long long)mx);
    __syncthreads();
    if (tid == 0) {
      const uint64_t old = thr[q];
      const uint64_t nt = ms->shmax < old ? (uint64_t)ms->shmax : old;
      thr[q] = nt;
      ms->shmax = nt;  // (the gate's threshold)
    }
    if (gate_cand != nullptr) {
      __syncthreads();
      select_gate(gate_cand, count, q, c, cap, ms->shmax, gate_num, gate_den, ms);
    }
  } else if (P2 <= 2 * kWave) {
    // k <= 128: one wave sorts the (at most 128) kept entries in registers,
    // two per lane (positions lane and lane + 64), the bitonic network of the
    // LDS sort below with shuffles instead of its 28 block barriers
    if (tid < kWave) {
      uint64_t a = tid < nres ? res[tid] : kEmpty;
      uint64_t b = tid + kWave < nres ? res[tid + kWave] : kEmpty;
      for (int size = 2; size <= 2 * kWave; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          if (stride == kWave) {  // partners in one lane; size 128: ascending
            const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
            a = lo;
            b = hi;
          } else {
            const uint64_t pa = shfl_xor_u64(a, stride), pb = shfl_xor_u64(b, stride);
            const bool lower = (tid & stride) == 0;
            const bool asc_a = (tid & size) == 0, asc_b = ((tid + kWave) & size) == 0;
            a = (lower == asc_a) ? (a < pa ? a : pa) : (a < pa ? pa : a);
            b = (lower == asc_b) ? (b < pb ? b : pb) : (b < pb ? pb : b);
          }
        }
      }
      const uint64_t e2[2] = {a, b};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int i = tid + h * kWave;
        if (i < k) {
          const uint64_t e = e2[h];
          out_dist[q * k + i] = e == kEmpty ? __builtin_nanf("") : key_float((uint32_t)(e >> 32));
          out_row[q * k + i] = e == kEmpty ? -1 : (int64_t)(e & 0xffffffffull);
        }
      }
    }
  } else {
    for (int i = nres + tid; i < P2; i += kSelectThreads) res[i] = kEmpty;
    __syncthreads();
    for (int size = 2; size <= P2; size <<= 1) {  // bitonic sort of res[0..P2)
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int i = tid; i < (P2 >> 1); i += kSelectThreads) {
          const int lo = (i / stride) * 2 * stride + (i % stride);
          const int hi = lo + stride;
          const bool asc = (lo & size) == 0;
          const uint64_t x = res[lo], y = res[hi];
          if ((x > y) == asc) {
            res[lo] = y;
            res[hi] = x;
          }
        }
        __syncthreads();
      }
    }
    for (int i = tid; i < k; i += kSelectThreads) {
      const uint64_t e = res[i];
      out_dist[q * k + i] = e == kEmpty ? __builtin_nanf("") : key_float((uint32_t)(e >> 32));
      out_row[q * k + i] = e == kEmpty ? -1 : (int64_t)(e & 0xffffffffull);
    }
  }
}

// The prune pass (select_kernel MODE 3): slices of kSelectEntries, used for
// k >= kPruneMinK when the buffer holds more than two slices (int8-image
// plans at k ~ 1 000: ~100 K candidates per query).  k-lists per query, 0 = off.
constexpr int kPruneMinK = 512;
int select_prune_lists(int64_t k, int64_t cap) {
  const int64_t o = option(kOptSelectPrune);
  if (o == 0 || (o == 1 && k < kPruneMinK) || cap <= 2 * (int64_t)kSelectEntries) return 0;
  return (int)((cap + kSelectEntries - 1) / kSelectEntries);
}

size_t select_prune_bytes(int64_t nq, int64_t k, int64_t cap) {
  return (size_t)nq * (size_t)select_prune_lists(k, cap) * (size_t)k * 8;
}

template <typename T, int MODE>
static int launch_select_one(const T* X, int64_t n, int d, int64_t row_base, const float* Q,
                             const float* qnorm, int64_t nq, const uint64_t* keys, int64_t cap,
                             uint32_t* count, int zero, int k, int metric, uint64_t* thr,
                             float* out_dist, int64_t* out_row, const uint64_t* alt,
                             int64_t alt_m, int64_t alt_gate, uint64_t* pre, int pre_p,
                             hipStream_t stream, const uint64_t* gate_cand = nullptr,
                             int64_t gate_num = 0, int64_t gate_den = 1) {
  const void* fn = metric == FX_METRIC_COS  ? (const void*)select_kernel<T, 2, MODE>
                   : metric == FX_METRIC_IP ? (const void*)select_kernel<T, 1, MODE>
                                            : (const void*)select_kernel<T, 0, MODE>;
  if (int rc = allow_lds(fn)) return rc;
  int P2 = 1;
  while (P2 < k) P2 <<= 1;
  const size_t smem = sizeof(MergeShared) + ((size_t)P2 + kSelectEntries) * 8;
  const int64_t pre_s = kSelectEntries;
  const unsigned gx = MODE == 3 ? (unsigned)pre_p : 1u;
  for (int64_t q0 = 0; q0 < nq; q0 += 65535) {
    const int64_t qn = (nq - q0) < 65535 ? (nq - q0) : 65535;
    const T* x = X;
    const float* qv = Q != nullptr ? Q + q0 * d : nullptr;
    const float* qnm = qnorm != nullptr ? qnorm + q0 : nullptr;
    const uint64_t* kq = keys + q0 * cap;
    uint32_t* cq = count + q0 * kCountStride;
    uint64_t* tq = thr != nullptr ? thr + q0 : nullptr;
    float* od = out_dist != nullptr ? out_dist + q0 * k : nullptr;
    int64_t* orow = out_row != nullptr ? out_row + q0 * k : nullptr;
    const uint64_t* aq = alt != nullptr ? alt + q0 * alt_m : nullptr;
    uint64_t* pq = pre != nullptr ? pre + q0 * (int64_t)pre_p * k : nullptr;
    const uint64_t* gq = gate_cand != nullptr ? gate_cand + q0 * cap : nullptr;
    void* args[] = {(void*)&x,   (void*)&n,     (void*)&d,     (void*)&row_base, (void*)&qv,
                    (void*)&qnm, (void*)&kq,    (void*)&cap,   (void*)&cq,       (void*)&zero,
                    (void*)&k,   (void*)&P2,    (void*)&tq,    (void*)&od,       (void*)&orow,
                    (void*)&aq,  (void*)&alt_m, (void*)&alt_gate, (void*)&pq,    (void*)&pre_p,
                    (void*)&pre_s, (void*)&gq, (void*)&gate_num, (void*)&gate_den};
    hipError_t e = hipLaunchKernel(fn, dim3(gx, (unsigned)qn), dim3(kSelectThreads), args, smem,
                                   stream);
    if (e != hipSuccess) {
      set_error("select_kernel launch: %s", hipGetErrorString(e));
      return FX_EHIP;
    }
  }
  return check_launch("select_kernel");
}

// One select (MODE 0/1/2); with a prune scratch (select_prune_bytes, may be
// null) and a plan that prunes (select_prune_lists), the MODE 3 pass first.
template <typename T, int MODE>
static int launch_select_t(const T* X, int64_t n, int d, int64_t row_base, const float* Q,
                           const float* qnorm, int64_t nq, const uint64_t* keys, int64_t cap,
                           uint32_t* count, int zero, int k, int metric, uint64_t* thr,
                           float* out_dist, int64_t* out_row, const uint64_t* alt,
                           int64_t alt_m, int64_t alt_gate, hipStream_t stream,
                           uint64_t* pre = nullptr, const uint64_t* gate_cand = nullptr,
                           int64_t gate_num = 0, int64_t gate_den = 1) {
  const int pre_p = pre != nullptr ? select_prune_lists(k, cap) : 0;
  if (pre_p == 0) pre = nullptr;
  if (pre != nullptr) {
    int rc = launch_select_one<T, 3>(X, n, d, row_base, Q, qnorm, nq, keys, cap, count, 0, k,
                                     metric, thr, out_dist, out_row, alt, alt_m, alt_gate, pre,
                                     pre_p, stream);
    if (rc) return rc;
  }
  return launch_select_one<T, MODE>(X, n, d, row_base, Q, qnorm, nq, keys, cap, count, zero, k,
                                    metric, thr, out_dist, out_row, alt, alt_m, alt_gate, pre,
                                    pre_p, stream, gate_cand, gate_num, gate_den);
}

int launch_exact_threshold(const void* X, int dtype, int64_t n, int d, int64_t row_base,
                           const float* Q, const float* qnorm, int64_t nq, const uint64_t* keys,
                           int64_t cap, uint32_t* count, bool zero_count, int k, int metric,
                           uint64_t* thr, hipStream_t stream, uint64_t* prune, int64_t* topr,
                           const uint64_t* gate_cand, int64_t gate_num, int64_t gate_den) {
  if (k > kSelectMaxK || k > cap) {
    set_error("exact threshold: k %d beyond cap %lld", k, (long long)cap);
    return FX_EUNSUPPORTED;
  }
  if (gate_cand != nullptr && (nq > 0x7fffffffll || gate_den <= 0 || zero_count)) {
    set_error("exact threshold gate: nq=%lld den=%lld zero=%d", (long long)nq,
              (long long)gate_den, (int)zero_count);
    return FX_EINVAL;
  }
  if (prune != nullptr && topr != nullptr && select_prune_lists(k, cap) > 0) {
    // large k: the pruned select writes the k rows, the chip rescores them
    // (one workgroup rescoring 1 000 rows of 3 KB took ~40 us of its time)
    int rc = dtype == FX_DTYPE_F16
                 ? launch_select_t<_Float16, 0>(reinterpret_cast<const _Float16*>(X), n, d,
                                                row_base, Q, qnorm, nq, keys, cap, count,
                                                zero_count ? 1 : 0, k, metric, thr, nullptr, topr,
                                                nullptr, 0, 0, stream, prune)
                 : launch_select_t<float, 0>(reinterpret_cast<const float*>(X), n, d, row_base, Q,
                                             qnorm, nq, keys, cap, count, zero_count ? 1 : 0, k,
                                             metric, thr, nullptr, topr, nullptr, 0, 0, stream,
                                             prune);
    if (rc) return rc;
    rc = launch_exact_kth(X, dtype, n, d, row_base, Q, qnorm, nq, k, topr, metric, thr, stream);
    if (rc || gate_cand == nullptr) return rc;
    return launch_overflow_gate(gate_cand, count, thr, nq, (int)cap, gate_num, gate_den, stream);
  }
  if (dtype == FX_DTYPE_F16)
    return launch_select_t<_Float16, 0>(reinterpret_cast<const _Float16*>(X), n, d, row_base, Q,
                                        qnorm, nq, keys, cap, count, zero_count ? 1 : 0, k, metric,
                                        thr, nullptr, nullptr, nullptr, 0, 0, stream, prune,
                                        gate_cand, gate_num, gate_den);
  return launch_select_t<float, 0>(reinterpret_cast<const float*>(X), n, d, row_base, Q, qnorm, nq,
                                   keys, cap, count, zero_count ? 1 : 0, k, metric, thr, nullptr,
                                   nullptr, nullptr, 0, 0, stream, prune, gate_cand, gate_num,
                                   gate_den);
}

int launch_sample_threshold(const uint64_t* keys, int64_t nq, int64_t cap, uint32_t* count,
                            bool zero_count, int k, uint64_t* thr, hipStream_t stream,
                            uint64_t* prune) {
  if (k > kSelectMaxK) {
    set_error("sample threshold: k %d too large", k);
    return FX_EUNSUPPORTED;
  }
  return launch_select_t<float, 2>(nullptr, 0, 1, 0, nullptr, nullptr, nq, keys, cap, count,
                                   zero_count ? 1 : 0, k, FX_METRIC_L2, thr, nullptr, nullptr,
                                   nullptr, 0, 0, stream, prune);
}

int launch_final_select(const uint64_t* keys, int64_t nq, int64_t cap, const uint32_t* count,
                        int k, float* out_dist, int64_t* out_row, const uint64_t* alt,
                        int64_t alt_m, int64_t alt_gate, hipStream_t stream, uint64_t* prune) {
  if (k > kSelectMaxK) {
    set_error("final select: k %d too large", k);
    return FX_EUNSUPPORTED;
  }
  // (MODE 1 reads no rows: the keys are exact composites already)
  return launch_select_t<float, 1>(nullptr, 0, 1, 0, nullptr, nullptr, nq, keys, cap,
                                   const_cast<uint32_t*>(count), 0, k, FX_METRIC_L2, nullptr,
                                   out_dist, out_row, alt, alt_m, alt_gate, stream, prune);
}

}  // namespace fx
