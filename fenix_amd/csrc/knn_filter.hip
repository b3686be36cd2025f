// Batched-query candidate filter on the fp16 matrix cores.
//
// configs[2] (10M x 768 f32 cosine, 256 queries) is a dense GEMM S = X . Q^T
// (reference: 256 separate per-chunk UDF searches, src/fenix/io/index/
// index.py:137-162 -> src/fenix/io/coder/coder.py:42-48).  On fp32 MFMA it is
// compute-bound (3.93 TFLOP at 157 TF/s = 25 ms).  This kernel evaluates the
// GEMM on the fp16 matrix cores (16x the rate), where one pass over the f32
// corpus is HBM-bound again, and uses each product only as a FILTER: with a
// rigorous bound e on |fp16 estimate - the single-query scan's f32 distance|
// every (row, query) gets an interval [lb, ub] that contains the distance the
// scan computes.  Rows are kept when lb can reach the query's threshold, and
// every kept candidate is rescored exactly (knn_batch.hip rescore_kernel: the
// scan's own summation order) before a result is taken.  No precision is given
// up: the returned distances and rows are bit-identical to the f32 scan.
//
// Error bound (u = 2^-11 fp16 unit roundoff, g = 2^-24):
//   x_i -> fp16: |dx_i| <= u |x_i| + 2^-14 (normal range; the absolute term
//   also covers subnormals flushed to zero); q is scaled by a power of two so
//   that max|q_i| lies in [2^14, 2^15) before rounding, |dq_i| <= u |q_i| +
//   2^-26 max|q|; fp16 x fp16 products are exact in fp32; the fp32 sums of the
//   estimate and of the scan are each within (d + 2) g sum|x_i q_i|.  Hence
//     |dot_est - dot_scan| <= (2u + u^2 + 2^-26 sqrt(d) + (4d + 16) g) |x||q|
//                             + 2^-14 sqrt(d) |q|
//   and per metric (slack 1.25 for the roundings of the bound itself):
//     IP   e = A |x| + B                 (A, B carry |q|)
//     L2   e = A (|x|^2 + |q|^2) + B     on the squared distance (the scan's
//          direct sum of (x - q)^2 is within 2 (d + 2) g of it; covered)
//     cos  e = A + B / max(|x|, 1e-12)   on 0.5 - 0.5 cos
//   Rows with a component of magnitude >= 65504 (fp16 overflow), a non-finite
//   sum of squares, or a query with non-finite norm are forced through
//   (lb = -inf, ub = NaN, i.e. above every number).
//
// Tile: 128 corpus rows x 256 queries per 512-thread workgroup (8 waves: 2 row
// groups x 4 query groups of 64; each wave holds 2 x 2 accumulators of
// v_mfma_f32_32x32x16_f16, 64 registers, so two waves share a SIMD).  K chunks
// of 64 elements: the f32 rows are loaded with non-temporal 16-B loads two
// chunks ahead (64 KB in flight per CU), converted to fp16 on the way into a
// double-buffered LDS tile (rows padded to 144 B: conflict-free ds_read_b128
// fragments); the pre-scaled fp16 query tile (L2-resident, 393 KB for
// 256 x 768) is staged alongside.  Per-row sums of squares and max |x| come
// from the same registers.
#include "fx_internal.h"
#include "fx_wave.h"

namespace fx {

constexpr int fBM = 128;                        // corpus rows per tile
constexpr int fBQ = 256;                        // queries per block
constexpr int fBK = 64;                         // K chunk (elements)
constexpr int fLds = fBK + 8;                   // padded LDS row (halves): 144 B
constexpr int fThreads = 512;                   // 8 waves: 2 row groups x 4 query groups of 64
constexpr int fXC = fBK / 4;                    // 16-B f32 pieces per row per chunk
constexpr int fQC = fBK / 8;                    // 16-B f16 pieces per query per chunk
constexpr int fXP = fBM * fXC / fThreads;       // X pieces per thread per chunk: 4
constexpr int fQP = fBQ * fQC / fThreads;       // Q pieces per thread per chunk: 4
constexpr int fRowLanes = fXC;                  // lanes sharing one row's pieces

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

struct FilterShared {
  _Float16 xs[2][fBM * fLds];
  _Float16 qs[2][fBQ * fLds];
  float rinfo[fBM];  // per-row bound factor (see the epilogue)
};

struct FilterPre {  // one chunk of X rows in flight (two of these: two chunks ahead)
  f32x4 x[fXP];
};
struct FilterPreQ {  // one chunk of the (L2-resident) query tile: one chunk ahead
  i32x4 q[fQP];
};

// Buffer loads: a per-tile descriptor (its size clips rows past n to zero) and
// 32-bit per-lane offsets, the chunk offset in the scalar operand.
struct FilterAddr {
  __amdgpu_buffer_rsrc_t xr, qr;
  int d, dq;
};

__device__ __forceinline__ void filter_load(FilterPre& p, const FilterAddr& ad, unsigned tid, int c) {
  const int k0 = c * fBK;
  const unsigned c4 = tid % fXC;                  // this lane's 16-B piece of a row chunk
  const bool in_row = k0 + (int)c4 * 4 < ad.d;   // past the row end: an offset beyond the buffer
#pragma unroll
  for (int i = 0; i < fXP; ++i) {
    const uint32_t off = (((i * fThreads + tid) / fXC) * (unsigned)ad.d + c4 * 4) * 4;
    p.x[i] = __builtin_bit_cast(
        f32x4, __builtin_amdgcn_raw_buffer_load_b128(ad.xr, in_row ? off : 0x7fff0000u, k0 * 4,
                                                     2 /* nt */));
  }
}

__device__ __forceinline__ void filter_load_q(FilterPreQ& p, const FilterAddr& ad, unsigned tid, int c) {
#pragma unroll
  for (int i = 0; i < fQP; ++i) {
    const uint32_t off = (((i * fThreads + tid) / fQC) * (unsigned)ad.dq + (tid % fQC) * 8) * 2;
    p.q[i] = __builtin_bit_cast(
        i32x4, __builtin_amdgcn_raw_buffer_load_b128(ad.qr, off, c * fBK * 2, 0));
  }
}

__device__ __forceinline__ void filter_store(const FilterPre& p, const FilterPreQ& pq,
                                             FilterShared* sh, int buf, unsigned tid,
                                             float (&sq)[fXP], float (&mx)[fXP]) {
#pragma unroll
  for (int i = 0; i < fXP; ++i) {
    const unsigned idx = i * fThreads + tid;
    const f32x4 v = p.x[i];
    *reinterpret_cast<f16x4*>(&sh->xs[buf][(idx / fXC) * fLds + (idx % fXC) * 4]) =
        __builtin_convertvector(v, f16x4);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sq[i] = fmaf(v[t], v[t], sq[i]);
      mx[i] = fmaxf(mx[i], fabsf(v[t]));
    }
  }
#pragma unroll
  for (int i = 0; i < fQP; ++i) {
    const unsigned idx = i * fThreads + tid;
    *reinterpret_cast<i32x4*>(&sh->qs[buf][(idx / fQC) * fLds + (idx % fQC) * 8]) = pq.q[i];
  }
}

// Hide a value from loop-invariant code motion: addresses derived from it are
// recomputed (a few VALU ops) where they are used instead of being hoisted out
// of the chunk loop and kept live (or spilled) across it.
__device__ __forceinline__ unsigned opaque(unsigned v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ __forceinline__ void filter_compute(f32x16 (&acc)[2][2], const FilterShared* sh,
                                               int buf, unsigned tid) {
  const unsigned lane = tid & 63, wid = tid >> 6;
  const unsigned rg = wid & 1, qg = wid >> 1, h = lane >> 5, l32 = lane & 31;
  const _Float16* xs = sh->xs[buf] + (rg * 64 + l32) * fLds + 8 * h;
  const _Float16* qs = sh->qs[buf] + (qg * 64 + l32) * fLds + 8 * h;
#pragma unroll
  for (int s = 0; s < fBK / 16; ++s) {
    f16x8 av[2], bv[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) av[t] = *reinterpret_cast<const f16x8*>(xs + t * 32 * fLds + 16 * s);
#pragma unroll
    for (int u = 0; u < 2; ++u) bv[u] = *reinterpret_cast<const f16x8*>(qs + u * 32 * fLds + 16 * s);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < 2; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[t], bv[u], acc[t][u], 0, 0, 0);
  }
}

template <int METRIC>
__global__ void __launch_bounds__(fThreads, 2) filter_kernel(FilterArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  FilterShared* sh = reinterpret_cast<FilterShared*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int rg = wid & 1, qg = wid >> 1;  // 64-row group, 64-query group
  const int h = lane >> 5, l32 = lane & 31;
  const int64_t q0 = (int64_t)blockIdx.y * fBQ;
  const int nch = (a.d + fBK - 1) / fBK;
  const int diag = a.diag;

  for (int64_t ti = blockIdx.x; ti < a.num_tiles; ti += gridDim.x) {
    const int64_t tile = a.tile_start + ti * a.tile_stride;
    const int64_t r0 = tile * fBM;
    if (r0 >= a.n) continue;

    f32x16 acc[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < 2; ++u) acc[t][u] = f32x16(0.f);
    float sq[fXP], mx[fXP];
#pragma unroll
    for (int i = 0; i < fXP; ++i) sq[i] = mx[i] = 0.f;

    const int64_t rows = a.n - r0 < fBM ? a.n - r0 : fBM;
    FilterAddr ad;
    {
      const float* xb = a.X + r0 * (int64_t)a.d;
      const uint64_t xp = reinterpret_cast<uint64_t>(xb);
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)xp);
      const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(xp >> 32));
      const int nb = __builtin_amdgcn_readfirstlane((int)(rows * a.d * 4));
      ad.xr = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
      const uint16_t* qb = a.Qh + q0 * (int64_t)a.dq;
      const uint64_t qp = reinterpret_cast<uint64_t>(qb);
      const uint32_t qlo = __builtin_amdgcn_readfirstlane((uint32_t)qp);
      const uint32_t qhi = __builtin_amdgcn_readfirstlane((uint32_t)(qp >> 32));
      const int qnb = __builtin_amdgcn_readfirstlane(fBQ * a.dq * 2);
      ad.qr = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<void*>(((uint64_t)qhi << 32) | qlo), 0, qnb, 0x00020000);
      ad.d = a.d;
      ad.dq = a.dq;
    }

    // X: two register stages (chunks c + 2 and c + 3 in flight while chunk c is
    // multiplied); Q (L2 hits): one stage.  Loads are issued unconditionally
    // (chunks past the row end read as zeros through the descriptor bounds):
    // a load under a branch makes the compiler wait for it where the branch
    // joins, which would drain the pipeline every chunk.  Q is issued before
    // X: waiting for Q(c + 2) next iteration must not wait for X(c + 3)
    // (vmcnt retires loads in issue order).
    FilterPre p0, p1;
    FilterPreQ pq;
    filter_load(p0, ad, opaque(tid), 0);
    filter_load_q(pq, ad, opaque(tid), 0);
    filter_load(p1, ad, opaque(tid), 1);
    filter_store(p0, pq, sh, 0, opaque(tid), sq, mx);
    filter_load_q(pq, ad, opaque(tid), 1);
    filter_load(p0, ad, opaque(tid), 2);
    __syncthreads();
    for (int c = 0; c < nch; c += 2) {
      if (!(diag & 4)) filter_compute(acc, sh, 0, opaque(tid));
      if (c + 1 < nch) filter_store(p1, pq, sh, 1, opaque(tid), sq, mx);
      filter_load_q(pq, ad, opaque(tid), c + 2);
      filter_load(p1, ad, opaque(tid), c + 3);
      __syncthreads();
      if (c + 1 >= nch) break;
      if (!(diag & 4)) filter_compute(acc, sh, 1, opaque(tid));
      if (c + 2 < nch) filter_store(p0, pq, sh, 0, opaque(tid), sq, mx);
      filter_load_q(pq, ad, opaque(tid), c + 3);
      filter_load(p0, ad, opaque(tid), c + 4);
      __syncthreads();
    }

    // per-row bound factor from |x|^2 and max|x| (the fRowLanes lanes of a row
    // hold partials): rinfo = the metric's row term, NaN = forced through
    // (fp16 overflow, non-finite), -1 = skipped (past n or masked out)
#pragma unroll
    for (int i = 0; i < fXP; ++i) {
#pragma unroll
      for (int m = 1; m < fRowLanes; m <<= 1) {
        sq[i] += __shfl_xor(sq[i], m);
        mx[i] = fmaxf(mx[i], __shfl_xor(mx[i], m));
      }
      if (tid % fRowLanes == 0) {
        const int lr = (i * fThreads + tid) / fXC;
        const int64_t row = r0 + lr;
        bool ok = row < a.n;
        if (ok && a.mask != nullptr) ok = (a.mask[row >> 5] >> (row & 31)) & 1u;
        float rterm;
        if constexpr (METRIC == 0) {
          rterm = sq[i];
        } else if constexpr (METRIC == 1) {
          rterm = sqrtf(sq[i]);
        } else {
          rterm = 1.f / fmaxf(sqrtf(sq[i]), 1e-12f);
        }
        if (!(mx[i] < 65504.f) || !(sq[i] <= 3.4e38f)) rterm = __builtin_nanf("");
        sh->rinfo[lr] = ok ? rterm : -1.f;
      }
    }
    __syncthreads();

    // ---- epilogue: [lb, ub] per (row, query), threshold test, append
    if (diag & 2) {
      if (acc[0][0][0] == 1.2345f && acc[1][1][5] == 2.f) a.count[0] = 7;
      continue;
    }
    // Pass test per (row, query) in a few fused ops on a conservative form of
    // lb <= threshold (extra passes only cost a rescored candidate); the lane's
    // passes over its 32 rows are collected in a bit mask per query column.
    // Forced rows (NaN row term) and forced queries (A = inf) pass by NaN/-inf.
    const int lr0 = rg * 64 + 4 * h;
    const float* ri = sh->rinfo + lr0;
    uint32_t pm[2];
    float qc1[2], qc0[2], qA[2], qB[2], qthr[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t gq = q0 + qg * 64 + u * 32 + l32;
      const bool live = gq < a.nq;
      const f32x4 info = live ? *reinterpret_cast<const f32x4*>(a.qinfo + gq * 4) : f32x4(0.f);
      const float tf = live ? key_float((uint32_t)(a.thr[gq] >> 32)) : -__builtin_inff();
      qA[u] = info[2];
      qB[u] = info[3];
      if constexpr (METRIC == 0) {
        qc1[u] = -2.f * info[0];
        qc0[u] = info[1];
        qthr[u] = tf * tf * (1.f + 9.5367431640625e-07f);  // lb <= T  <=  lb^2 <= T^2 (1 + 2^-20)
      } else if constexpr (METRIC == 1) {
        qc1[u] = -info[0];
        qthr[u] = tf;
      } else {
        qc1[u] = -0.5f * info[0] / info[1];
        qthr[u] = tf;
      }
      pm[u] = 0u;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int off = t * 32 + (r & 3) + 8 * (r >> 2);  // compile-time row offset
          const float rterm = ri[off];
          const float x = acc[t][u][r];
          float v;
          if constexpr (METRIC == 0) {
            const float s2 = rterm + qc0[u];
            v = fmaf(x, qc1[u], s2) - fmaf(qA[u], s2, qB[u]);
          } else if constexpr (METRIC == 1) {
            v = fmaf(x, qc1[u], -fmaf(qA[u], rterm, qB[u]));
          } else {
            v = fmaf(x * rterm, qc1[u], 0.5f) - fmaf(qB[u], rterm, qA[u]);
          }
          // rterm < 0: skipped row (past n / masked out); NaN v passes
          const bool pass = !(v > qthr[u]) && !(rterm < 0.f);
          pm[u] |= (uint32_t)pass << (t * 16 + r);
        }
      }
      if (!live || (diag & 1)) pm[u] = 0u;
    }
    // one atomic per (lane, query column) with passes: positions for all of them
    uint32_t pos[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      pos[u] = 0u;
      if (pm[u] != 0u) {
        const int64_t gq = q0 + qg * 64 + u * 32 + l32;
        pos[u] = atomicAdd(&a.count[gq * kCountStride], (uint32_t)__popc(pm[u]));
      }
    }
    if (__ballot((pm[0] | pm[1]) != 0u) == 0ull) continue;
    const uint32_t grow0 = (uint32_t)(a.row_base + r0 + lr0);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t gq = q0 + qg * 64 + u * 32 + l32;
      const bool fq = !(qA[u] <= 3.4e38f);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (!((pm[u] >> (t * 16 + r)) & 1u)) continue;
          const int off = t * 32 + (r & 3) + 8 * (r >> 2);
          const float rterm = ri[off];
          const float x = acc[t][u][r];
          float lb, ub;
          if constexpr (METRIC == 0) {
            const float s2 = rterm + qc0[u];
            const float d2 = fmaf(x, qc1[u], s2);
            const float e = fmaf(qA[u], s2, qB[u]);
            lb = sqrtf(fmaxf(d2 - e, 0.f));
            ub = sqrtf(d2 + e);
          } else if constexpr (METRIC == 1) {
            const float e = fmaf(qA[u], rterm, qB[u]);
            lb = fmaf(x, qc1[u], -e);
            ub = fmaf(x, qc1[u], e);
          } else {
            const float dist = fmaf(x * rterm, qc1[u], 0.5f);
            const float e = fmaf(qB[u], rterm, qA[u]);
            lb = dist - e;
            ub = dist + e;
          }
          if (fq || rterm != rterm) {  // forced: below / above every key
            lb = -__builtin_inff();
            ub = __builtin_nanf("");
          }
          const uint32_t p = pos[u]++;
          if (p < (uint32_t)a.cap) {
            const uint32_t grow = grow0 + (uint32_t)off;
            const size_t slot = (size_t)gq * a.cap + p;
            if (a.cand_ub != nullptr) {
              a.cand[slot] = make_comp(lb, grow);
              a.cand_ub[slot] = make_comp(ub, grow);
            } else {
              a.cand[slot] = make_comp(ub, grow);
            }
          }
        }
      }
    }
  }
}

int launch_filter(const FilterArgs& a, int metric, hipStream_t stream) {
  if (a.num_tiles <= 0) return FX_OK;
  const size_t smem = sizeof(FilterShared);
  const void* fn = metric == FX_METRIC_COS ? (const void*)filter_kernel<2>
                   : metric == FX_METRIC_IP ? (const void*)filter_kernel<1>
                                            : (const void*)filter_kernel<0>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)filter_kernel<2>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    (void)hipFuncSetAttribute((const void*)filter_kernel<1>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    (void)hipFuncSetAttribute((const void*)filter_kernel<0>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr = true;
  }
  int cus = 0;
  int rc = device_cus(&cus);
  if (rc) return rc;
  const int64_t qtiles = (a.nq + fBQ - 1) / fBQ;
  int64_t bx = cus;
  if (bx > a.num_tiles) bx = a.num_tiles;
  for (int64_t y0 = 0; y0 < qtiles; y0 += 65535) {
    FilterArgs b = a;
    const int64_t yn = (qtiles - y0) < 65535 ? (qtiles - y0) : 65535;
    b.Qh = a.Qh + y0 * fBQ * (int64_t)a.dq;
    b.qinfo = a.qinfo + y0 * fBQ * 4;
    b.thr = a.thr + y0 * fBQ;
    b.count = a.count + y0 * fBQ * kCountStride;
    b.cand = a.cand + y0 * fBQ * (int64_t)a.cap;
    if (a.cand_ub) b.cand_ub = a.cand_ub + y0 * fBQ * (int64_t)a.cap;
    b.nq = a.nq - y0 * fBQ;
    void* args[] = {(void*)&b};
    hipError_t e = hipLaunchKernel(fn, dim3((unsigned)bx, (unsigned)yn), dim3(fThreads), args,
                                   smem, stream);
    if (e != hipSuccess) {
      set_error("filter_kernel launch: %s", hipGetErrorString(e));
      return FX_EHIP;
    }
  }
  return check_launch("filter_kernel");
}

int filter_tile_rows() { return fBM; }
int filter_query_pad() { return fBQ; }
int filter_dq(int d) { return (d + fBK - 1) / fBK * fBK; }

// Per query: the fp16 image scaled by 2^s (max|q| in [2^14, 2^15)), zero-padded
// to dq halves, and the bound constants {2^-s, norm term, A, B} (see the
// header).  The norm term is the scan's: sum of squares in the scan's order
// (lane-strided fmaf chain + xor butterfly, knn_scan.hip) -> |q|^2 (L2),
// |q| (IP), max(|q|, 1e-12) (cosine, coder.py:43-44).  Queries beyond nq
// (up to the padded count) are zero.  One wave per query.
__global__ void qprep_kernel(const float* __restrict__ Q, int64_t nq, int64_t nq_pad, int d, int dq,
                             int metric, uint16_t* __restrict__ Qh, float* __restrict__ qinfo) {
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (q >= nq_pad) return;
  _Float16* out = reinterpret_cast<_Float16*>(Qh) + q * (int64_t)dq;
  if (q >= nq) {
    for (int i = lane; i < dq; i += 64) out[i] = (_Float16)0.f;
    return;
  }
  const float* qv = Q + q * (int64_t)d;
  float s = 0.f, m = 0.f;
  for (int i = lane; i < d; i += 64) {
    s = fmaf(qv[i], qv[i], s);
    m = fmaxf(m, fabsf(qv[i]));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    s += __shfl_xor(s, o);
    m = fmaxf(m, __shfl_xor(m, o));
  }
  // power-of-two scale: exact, so the fp16 rounding is the only query error
  int ex = 0;
  if (m > 0.f && m <= 3.4e38f) (void)frexpf(m, &ex);  // m in [2^(ex-1), 2^ex)
  const int sh = 15 - ex;
  const float scale = ldexpf(1.f, sh > 126 ? 126 : (sh < -126 ? -126 : sh));
  for (int i = lane; i < dq; i += 64) out[i] = (_Float16)(i < d ? qv[i] * scale : 0.f);
  if (lane == 0) {
    const double u = 1.0 / 2048.0, g = 5.9604644775390625e-08;
    const double sd = sqrt((double)d);
    const double rel = 1.25 * (2.0 * u + u * u + sd * 1.4901161193847656e-08 + (4.0 * d + 16.0) * g);
    const double abs_ = 1.25 * sd * 6.103515625e-05 * (1.0 + 1.0 / 1024.0);
    const float qn = sqrtf(s);
    float a, b, t;
    if (metric == FX_METRIC_L2) {
      t = s;
      a = (float)rel;
      b = (float)(2.0 * abs_ * (double)qn);
    } else if (metric == FX_METRIC_IP) {
      t = qn;
      a = (float)(rel * (double)qn);
      b = (float)(abs_ * (double)qn);
    } else {
      t = fmaxf(qn, 1e-12f);
      a = (float)(0.5 * rel);
      b = (float)(0.5 * abs_);
    }
    if (!(s <= 3.4e38f) || !(m <= 3.4e38f)) a = __builtin_inff();  // forced query
    float* info = qinfo + q * 4;
    info[0] = 1.f / scale;
    info[1] = t;
    info[2] = a;
    info[3] = b;
  }
}

int launch_qprep(const float* Q, int64_t nq, int64_t nq_pad, int d, int dq, int metric,
                 uint16_t* Qh, float* qinfo, hipStream_t stream) {
  hipLaunchKernelGGL(qprep_kernel, dim3((unsigned)((nq_pad + 3) / 4)), dim3(256), 0, stream, Q,
                     nq, nq_pad, d, dq, metric, Qh, qinfo);
  return check_launch("qprep_kernel");
}

}  // namespace fx
