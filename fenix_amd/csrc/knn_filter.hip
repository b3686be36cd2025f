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
//   A component of magnitude >= 65520 (rounds to an fp16 infinity, so the
//   product comes out non-finite), a non-finite sum of squares or a query with
//   a non-finite norm forces the pair through (lb = -inf, ub = NaN, i.e. above
//   every number).  Components in [65504, 65520) round to 65504 within u.
//
// Tile: 256 corpus rows x 256 queries per 512-thread workgroup, one per CU
// (8 waves, 2 per SIMD: 4 row groups of 64 x 2 query groups of 128; each wave
// holds 2 x 4 accumulators of v_mfma_f32_32x32x16_f16).  K chunks of 32: the
// f32 rows stream in through buffer loads (non-temporal) two chunks ahead,
// are converted to fp16 on their way into a double-buffered LDS tile (rows
// padded by 16 B: conflict-free ds_read_b128 fragments); the pre-scaled fp16
// query tile (L2-resident, 393 KB for 256 x 768) is staged alongside, one
// chunk ahead.  Per-row sums of squares and fp16-overflow flags come from the
// same registers.  Measured (10M x 768, 256 queries, tools/filter_diag.py):
// the X stream alone runs at 6.8 TB/s; re-reading the query tile from L2 for
// every 256-row tile and the LDS staging cost ~1.3 ms of a ~6 ms pass, the
// MFMAs (16 % of the fp16 peak) ~1 ms, the epilogue ~0.6 ms.
#include "fx_internal.h"
#include "fx_wave.h"

namespace fx {

#ifndef FX_FILTER_WAVES
#define FX_FILTER_WAVES 8   // waves per workgroup (two per SIMD)
#endif
#ifndef FX_FILTER_BPC
#define FX_FILTER_BPC 1     // workgroups per CU (LDS and registers permitting)
#endif
#ifndef FX_FILTER_STAGES
#define FX_FILTER_STAGES 2  // K chunks of X in flight per thread
#endif
#ifndef FX_FILTER_BM
#define FX_FILTER_BM 256
#endif
#ifndef FX_FILTER_BK
#define FX_FILTER_BK 32
#endif
constexpr int fBM = FX_FILTER_BM;               // corpus rows per tile
constexpr int fBQ = 256;                        // queries per block
constexpr int fBK = FX_FILTER_BK;               // K chunk (elements)
constexpr int fLds = fBK + 8;                   // padded LDS row (halves): 16 B pad
constexpr int fWaves = FX_FILTER_WAVES;
constexpr int fThreads = 64 * fWaves;           // waves: fRG row groups x fQG query groups
constexpr int fRG = fBM / 64;                   // 64-row groups (2 MFMA row tiles each)
constexpr int fQG = fWaves / fRG;               // query groups
constexpr int fQT = fBQ / fQG / 32;             // 32-query MFMA tiles per wave
constexpr int fStages = FX_FILTER_STAGES;
constexpr int fXC = fBK / 4;                    // 16-B f32 pieces per row per chunk
constexpr int fQC = fBK / 8;                    // 16-B f16 pieces per query per chunk
constexpr int fXP = fBM * fXC / fThreads;       // X pieces per thread per chunk
constexpr int fQP = fBQ * fQC / fThreads;       // Q pieces per thread per chunk
constexpr int fRowLanes = fXC;                  // lanes sharing one row's pieces
static_assert(fQG >= 1 && fRG * fQG == fWaves && fQT >= 1, "wave grid");
static_assert(fXP >= 1 && fQP >= 1 && fBK % 16 == 0, "staging");

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

struct FilterShared {
  _Float16 xs[2][fBM * fLds];
  _Float16 qs[2][fBQ * fLds];
  float rinfo[fBM];  // per-row bound factor (see the epilogue)
  f32x4 qtab[fBQ];   // per query: the bound's constants {c1, c0, A, B}
  float2 qab[fBQ];   // per query: pass iff product >= a * row value + b
};

struct FilterPre {  // one K chunk of X rows in flight
  f32x4 x[fXP];
};
struct FilterPreQ {  // one K chunk of the (L2-resident) query tile
  i32x4 q[fQP];
};

// Buffer loads: a per-tile descriptor (its size clips rows past n to zero) and
// 32-bit per-lane offsets, the chunk offset in the scalar operand.
struct FilterAddr {
  __amdgpu_buffer_rsrc_t xr, qr;
  int d, dq;
};

__device__ __forceinline__ void filter_load_q(FilterPreQ& p, const FilterAddr& ad, unsigned tid,
                                              int c, int diag) {
#pragma unroll
  for (int i = 0; i < fQP; ++i) {
    if (diag & 8) {
      p.q[i] = i32x4(0);
      continue;
    }
    const uint32_t off = (((i * fThreads + tid) / fQC) * (unsigned)ad.dq + (tid % fQC) * 8) * 2;
    p.q[i] = __builtin_bit_cast(
        i32x4, __builtin_amdgcn_raw_buffer_load_b128(ad.qr, off, c * fBK * 2, 0));
  }
}

__device__ __forceinline__ void filter_load(FilterPre& p, const FilterAddr& ad, unsigned tid, int c) {
  const int k0 = c * fBK;
  const unsigned c4 = tid % fXC;                 // this lane's 16-B piece of a row chunk
  const bool in_row = k0 + (int)c4 * 4 < ad.d;  // past the row end: an offset beyond the buffer
#pragma unroll
  for (int i = 0; i < fXP; ++i) {
    const uint32_t off = (((i * fThreads + tid) / fXC) * (unsigned)ad.d + c4 * 4) * 4;
    p.x[i] = __builtin_bit_cast(
        f32x4, __builtin_amdgcn_raw_buffer_load_b128(ad.xr, in_row ? off : 0x7fff0000u, k0 * 4,
                                                     2 /* nt */));
  }
}

__device__ __forceinline__ void filter_store(const FilterPre& p, const FilterPreQ& pq,
                                             FilterShared* sh, int buf, unsigned tid,
                                             float (&sq)[fXP], uint32_t& ovf) {
#pragma unroll
  for (int i = 0; i < fXP; ++i) {
    const unsigned idx = i * fThreads + tid;
    const f32x4 v = p.x[i];
    *reinterpret_cast<f16x4*>(&sh->xs[buf][(idx / fXC) * fLds + (idx % fXC) * 4]) =
        __builtin_convertvector(v, f16x4);
#pragma unroll
    for (int t = 0; t < 4; ++t) sq[i] = fmaf(v[t], v[t], sq[i]);
    // a component that rounds to an fp16 infinity (|x| >= 65520)
    const float m = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
    ovf |= (uint32_t)(m >= 65520.f) << i;
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

__device__ __forceinline__ void filter_compute(f32x16 (&acc)[2][fQT], const FilterShared* sh,
                                               int buf, unsigned tid) {
  const unsigned lane = tid & 63, wid = tid >> 6;
  const unsigned rg = wid % fRG, qg = wid / fRG, h = lane >> 5, l32 = lane & 31;
  const _Float16* xs = sh->xs[buf] + (rg * 64 + l32) * fLds + 8 * h;
  const _Float16* qs = sh->qs[buf] + (qg * fQT * 32 + l32) * fLds + 8 * h;
#pragma unroll
  for (int s = 0; s < fBK / 16; ++s) {
    f16x8 av[2], bv[fQT];
#pragma unroll
    for (int t = 0; t < 2; ++t) av[t] = *reinterpret_cast<const f16x8*>(xs + t * 32 * fLds + 16 * s);
#pragma unroll
    for (int u = 0; u < fQT; ++u) bv[u] = *reinterpret_cast<const f16x8*>(qs + u * 32 * fLds + 16 * s);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < fQT; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[t], bv[u], acc[t][u], 0, 0, 0);
  }
}

template <int METRIC>
__global__ void __launch_bounds__(fThreads, fWaves * FX_FILTER_BPC / 4) filter_kernel(FilterArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  FilterShared* sh = reinterpret_cast<FilterShared*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int rg = wid % fRG, qg = wid / fRG;  // 64-row group, fQT*32-query group
  const int h = lane >> 5, l32 = lane & 31;
  const int64_t q0 = (int64_t)blockIdx.y * fBQ;
  const int nch = (a.d + fBK - 1) / fBK;
  const int diag = a.diag;

  // per-query constants (once per block).  The pass test lb <= T is linear in
  // the product x for a fixed row, so it is precomputed as x >= a * rv + b
  // with rv the row's value (cosine: max(|x|, 1e-12); IP: |x|; L2: |x|^2):
  //   cos  lb = x c1 / rv + 0.5 - A - B / rv,  c1 = -0.5 / (scale |q|) < 0
  //        -> x >= ((T - 0.5 + A) rv + B) / c1
  //   IP   lb = -x / scale - A rv - B           -> x >= (-T - B - A rv) scale
  //   L2   lb^2 = s2 - 2 x / scale - A s2 - B,  s2 = rv + |q|^2, against
  //        T^2 (1 + 2^-20) -> x >= ((1 - A) s2 - B - T^2) scale / 2
  // The roundings of this rearrangement are far inside the bound's slack.
  // T = NaN (no threshold yet) or a forced query: everything passes
  // (a = 0, b = -inf); padding queries: nothing (b = +inf).
  for (int i = tid; i < fBQ; i += fThreads) {
    const int64_t gq = q0 + i;
    f32x4 c = f32x4(0.f);
    float2 ab = {0.f, __builtin_inff()};
    if (gq < a.nq) {
      const f32x4 info = *reinterpret_cast<const f32x4*>(a.qinfo + gq * 4);
      const float tf = key_float((uint32_t)(a.thr[gq] >> 32));
      const float qinv = info[0], qa = info[1], qA = info[2], qB = info[3];
      c[2] = qA;
      c[3] = qB;
      if constexpr (METRIC == 0) {
        c[0] = -2.f * qinv;
        c[1] = qa;
        const float t2 = tf * tf * (1.f + 9.5367431640625e-07f);
        const float h = 0.5f / qinv;
        ab.x = (1.f - qA) * h;
        ab.y = ((1.f - qA) * qa - qB - t2) * h;
      } else if constexpr (METRIC == 1) {
        c[0] = -qinv;
        const float sc = 1.f / qinv;
        ab.x = -qA * sc;
        ab.y = (-tf - qB) * sc;
      } else {
        c[0] = -0.5f * qinv / qa;
        ab.x = (tf - 0.5f + qA) / c[0];
        ab.y = qB / c[0];
      }
      if (tf != tf || !(qA <= 3.4e38f)) ab = {0.f, -__builtin_inff()};
    }
    sh->qtab[i] = c;
    sh->qab[i] = ab;
  }
  // (the first tile's barriers order these writes before the epilogue reads)

  for (int64_t ti = blockIdx.x; ti < a.num_tiles; ti += gridDim.x) {
    const int64_t tile = a.tile_start + ti * a.tile_stride;
    const int64_t r0 = tile * fBM;
    if (r0 >= a.n) continue;

    f32x16 acc[2][fQT];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < fQT; ++u) acc[t][u] = f32x16(0.f);
    float sq[fXP];
#pragma unroll
    for (int i = 0; i < fXP; ++i) sq[i] = 0.f;
    uint32_t ovf = 0u;

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

    // fStages register stages: chunks c + 2 .. c + fStages of X and Q are in
    // flight while chunk c is multiplied (stage j % fStages holds chunk j).
    // Loads are issued unconditionally (chunks past the row end read as zeros
    // through the descriptor bounds): a load under a branch makes the compiler
    // wait for it where the branch joins, draining the pipeline every chunk.
    FilterPre pf[fStages];
    FilterPreQ pq;
#pragma unroll
    for (int j = 0; j < fStages; ++j) {
      if (j == 0) filter_load_q(pq, ad, opaque(tid), 0, diag);
      filter_load(pf[j], ad, opaque(tid), j);
    }
    filter_store(pf[0], pq, sh, 0, opaque(tid), sq, ovf);
    // Q one chunk ahead, issued before the X load of the same step: vmcnt
    // retires loads in issue order, so waiting for Q(c + 1) at step c waits
    // for X(c + 1) (needed there anyway) and nothing issued later.
    filter_load_q(pq, ad, opaque(tid), 1, diag);
    filter_load(pf[0], ad, opaque(tid), fStages);
    __syncthreads();
    for (int c0 = 0; c0 < nch; c0 += fStages) {
#pragma unroll
      for (int j = 0; j < fStages; ++j) {
        const int c = c0 + j;
        if (c >= nch) break;
        if (!(diag & 4)) filter_compute(acc, sh, c & 1, opaque(tid));
        if (c + 1 < nch && !(diag & 16))
          filter_store(pf[(j + 1) % fStages], pq, sh, (c + 1) & 1, opaque(tid), sq, ovf);
        filter_load_q(pq, ad, opaque(tid), c + 2, diag);
        filter_load(pf[(j + 1) % fStages], ad, opaque(tid), c + 1 + fStages);
        __syncthreads();
      }
    }

    // per-row value rv from |x|^2 (the fRowLanes lanes of a row hold partials):
    // cosine max(|x|, 1e-12), IP |x|, L2 |x|^2; NaN = forced through (fp16
    // overflow, non-finite); -1 = skipped (past n or masked out)
#pragma unroll
    for (int i = 0; i < fXP; ++i) {
#pragma unroll
      for (int m = 1; m < fRowLanes; m <<= 1) sq[i] += __shfl_xor(sq[i], m);
    }
#pragma unroll
    for (int m = 1; m < fRowLanes; m <<= 1) ovf |= __shfl_xor(ovf, m);
#pragma unroll
    for (int i = 0; i < fXP; ++i) {
      if (tid % fRowLanes == 0) {
        const int lr = (i * fThreads + tid) / fXC;
        const int64_t row = r0 + lr;
        bool ok = row < a.n;
        if (ok && a.mask != nullptr) ok = (a.mask[row >> 5] >> (row & 31)) & 1u;
        float rv;
        if constexpr (METRIC == 0) {
          rv = sq[i];
        } else if constexpr (METRIC == 1) {
          rv = sqrtf(sq[i]);
        } else {
          rv = fmaxf(sqrtf(sq[i]), 1e-12f);
        }
        if (!(sq[i] <= 3.4e38f) || ((ovf >> i) & 1u)) rv = __builtin_nanf("");
        sh->rinfo[lr] = ok ? rv : -1.f;
      }
    }
    __syncthreads();

    // ---- epilogue: [lb, ub] per (row, query), threshold test, append
    if (diag & 2) {
      if (acc[0][0][0] == 1.2345f && acc[1][fQT - 1][5] == 2.f) a.count[0] = 7;
      continue;
    }

    // Pass test: one fma and a compare per (row, query) (see the table above;
    // extra passes only cost a rescored candidate); the lane's passes over its
    // 32 rows are collected in a bit mask per query column, one atomic per
    // (lane, column) reserves their slots.  Forced rows always pass, skipped
    // rows never.
    const int lr0 = rg * 64 + 4 * h;
    const float* ri = sh->rinfo + lr0;
    const uint32_t grow0 = (uint32_t)(a.row_base + r0 + lr0);
    float rvs[32];
    uint32_t fmask = 0u, smask = 0u;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float rv = ri[t * 32 + (r & 3) + 8 * (r >> 2)];  // compile-time row offset
        rvs[t * 16 + r] = rv;
        fmask |= (uint32_t)(rv != rv) << (t * 16 + r);
        smask |= (uint32_t)(rv < 0.f) << (t * 16 + r);
      }
    }
    uint32_t pm[fQT];
#pragma unroll
    for (int u = 0; u < fQT; ++u) {
      const float2 ab = sh->qab[qg * fQT * 32 + u * 32 + l32];
      uint32_t m = 0u;
#pragma unroll
      for (int j = 0; j < 32; ++j)
        m |= (uint32_t)(acc[j >> 4][u][j & 15] >= fmaf(ab.x, rvs[j], ab.y)) << j;
      pm[u] = (diag & 1) ? 0u : ((m | fmask) & ~smask);
      if (q0 + qg * fQT * 32 + u * 32 + l32 >= a.nq) pm[u] = 0u;
    }
    uint32_t any = 0u;
#pragma unroll
    for (int u = 0; u < fQT; ++u) any |= pm[u];
    if (__ballot(any != 0u) == 0ull) continue;
    uint32_t pos[fQT];
#pragma unroll
    for (int u = 0; u < fQT; ++u) {
      pos[u] = 0u;
      const int64_t gq = q0 + qg * fQT * 32 + u * 32 + l32;
      if (pm[u] != 0u) pos[u] = atomicAdd(&a.count[gq * kCountStride], (uint32_t)__popc(pm[u]));
    }
#pragma unroll
    for (int u = 0; u < fQT; ++u) {
      if (__ballot(pm[u] != 0u) == 0ull) continue;
      const int qi = qg * fQT * 32 + u * 32 + l32;
      const int64_t gq = q0 + qi;
      const f32x4 qc = sh->qtab[qi];
      const float qc1 = qc[0], qc0 = qc[1], qA = qc[2], qB = qc[3];
      const bool fq = !(qA <= 3.4e38f);
      uint32_t p = pos[u];
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        if (!((pm[u] >> j) & 1u)) continue;
        const float rv = rvs[j];
        const float x = acc[j >> 4][u][j & 15];
        float lb, ub;
        if constexpr (METRIC == 0) {
          const float s2 = rv + qc0;
          const float d2 = fmaf(x, qc1, s2);
          const float e = fmaf(qA, s2, qB);
          lb = sqrtf(fmaxf(d2 - e, 0.f));
          ub = sqrtf(d2 + e);
        } else if constexpr (METRIC == 1) {
          const float e = fmaf(qA, rv, qB);
          lb = fmaf(x, qc1, -e);
          ub = fmaf(x, qc1, e);
        } else {
          const float rterm = 1.f / rv;
          const float dist = fmaf(x * rterm, qc1, 0.5f);
          const float e = fmaf(qB, rterm, qA);
          lb = dist - e;
          ub = dist + e;
        }
        if (fq || rv != rv) {  // forced: below / above every key
          lb = -__builtin_inff();
          ub = __builtin_nanf("");
        }
        if (p < (uint32_t)a.cap) {
          const uint32_t grow = grow0 + (uint32_t)(((j >> 4) * 32) + ((j & 15) & 3) + 8 * ((j & 15) >> 2));
          const size_t slot = (size_t)gq * a.cap + p;
          if (a.cand_ub != nullptr) {
            a.cand[slot] = make_comp(lb, grow);
            a.cand_ub[slot] = make_comp(ub, grow);
          } else {
            a.cand[slot] = make_comp(ub, grow);
          }
        }
        ++p;
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
  int64_t bx = (int64_t)cus * FX_FILTER_BPC;
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
