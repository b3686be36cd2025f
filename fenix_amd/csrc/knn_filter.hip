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
// same registers.  Measured (10M x 768, 256 queries: 8.5 ms per batch,
// tools/filter_diag.py switching parts off): the X stream alone runs at
// 6.8 TB/s (4.6 ms for all phases); re-reading the query tile from L2 for
// every 256-row tile and the LDS staging add ~1.3 ms, the MFMAs (~19 % of the
// dense fp16 peak, not overlapped with the stream inside one workgroup per
// CU) ~1 ms, the bound/test epilogue ~0.6 ms, the appends ~0.9 ms.  The
// 64-query variant: 4 row groups x 2 query groups of 32, K chunks of 64.
#include "fx_internal.h"
#include "fx_wave.h"

#include <type_traits>

// This file is compiled twice: as itself (256-query tiles, namespace
// fx::q256, plus the shared entry points) and through knn_filter_q64.hip
// (FX_FILTER_VARIANT: 64-query tiles, namespace fx::q64) and knn_filter_q128.hip
// (128-query tiles, fx::q128) for small batches,
// where a 256-query tile would re-read and multiply mostly padding.
#ifndef FX_FILTER_BQ
#define FX_FILTER_BQ 256
#endif
#ifndef FX_FILTER_ROWS  // row types compiled: 1 f32, 2 fp16
#define FX_FILTER_ROWS (FX_FILTER_BQ == 64 ? 3 : FX_FILTER_BK == 64 ? 2 : 1)
#endif
#ifndef FX_FILTER_IMPL
#define FX_FILTER_IMPL q256
#endif

namespace fx {
namespace FX_FILTER_IMPL {

#if !defined(FX_FILTER_VARIANT) && defined(FX_Q256_WAVES)  // knob of this compilation only
#define FX_FILTER_WAVES FX_Q256_WAVES
#endif
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
#define FX_FILTER_BK (FX_FILTER_BQ >= 256 ? 32 : 64)  // >= 1 query piece per thread
#endif
#ifndef FX_FILTER_IMG3  // the 256-query, 32-wide-K build (knn_filter.hip itself):
                        // filter_img3_kernel serves tiled filter images
#if FX_FILTER_BK == 32 && FX_FILTER_BQ >= 128
#define FX_FILTER_IMG3 1
#else
#define FX_FILTER_IMG3 0
#endif
#endif
constexpr int fBM = FX_FILTER_BM;               // corpus rows per tile
constexpr int fBQ = FX_FILTER_BQ;               // queries per block
constexpr int fBK = FX_FILTER_BK;               // K chunk (elements)
constexpr int fLds = fBK + 8;                   // padded LDS row (halves): 16 B pad
constexpr int fWaves = FX_FILTER_WAVES;
constexpr int fThreads = 64 * fWaves;           // waves: fRG row groups x fQG query groups
constexpr int fRG = fBM / 64;                   // 64-row groups (2 MFMA row tiles each)
constexpr int fQG = fWaves / fRG;               // query groups
constexpr int fQT = fBQ / fQG / 32;             // 32-query MFMA tiles per wave
constexpr int fStages = FX_FILTER_STAGES;
// Cross-tile prefetch (see filter_tiles): measured faster for the 64-query
// tiles (16 queries, 10M x 768 image: 2.73 -> 2.65 ms), slower for the
// 256-query ones (5.99 -> 6.1 ms BK 32, 6.35 ms BK 64: register pressure)
#ifndef FX_FILTER_XPF
#define FX_FILTER_XPF (FX_FILTER_BQ == 64)
#endif
constexpr bool kXpf = FX_FILTER_XPF;
static_assert(fStages == 2, "the K loop alternates two register stages and two LDS buffers");
constexpr int fQC = fBK / 8;                    // 16-B f16 pieces per query per chunk
// Q pieces per thread per chunk (a build with no register-staged kernels,
// FX_FILTER_ROWS 0, may have fewer pieces than threads)
constexpr int fQP = fBQ * fQC / fThreads > 0 ? fBQ * fQC / fThreads : 1;
// Rows of type XT (float or _Float16) come in 16-B pieces of E elements;
// C pieces per row per chunk (the lanes sharing a row), P per thread.
template <typename XT>
struct XPiece {
  static constexpr int E = 16 / (int)sizeof(XT);
  static constexpr int C = fBK / E;
  static constexpr int P = fBM * C / fThreads;
  static_assert(P >= 1 && fThreads % C == 0, "row staging");
};
static_assert(fQG >= 1 && fRG * fQG == fWaves && fQT >= 1, "wave grid");
static_assert((FX_FILTER_ROWS == 0 || fBQ * fQC / fThreads >= 1) && fBK % 16 == 0, "staging");

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// Per-tile row flags for the epilogue, by tile parity: [forced | skipped][8]
// 32-bit masks, one per (64-row group, lane half) in the bit order of the
// lane's accumulator rows (filter_row_bit); up to 16 (row group, lane half)
// words per kind: 32-row groups (the tiled-image kernel) or 64-row groups
constexpr int kRowFlagWords = 2 * 16;
static_assert(fBM <= 256, "row flag words: (64-row group, lane half) <= 8");
struct FilterShared {
  _Float16 xs[2][fBM * fLds];
  _Float16 qs[2][fBQ * fLds];
  float rinfo[fBM];  // per-row bound factor (see the epilogue)
  float rterm[fBM];  // cosine: 1 / rinfo (the appends' bound term)
  uint32_t rflags[2][kRowFlagWords];
  f32x4 qtab[fBQ];   // per query: the bound's constants {c1, c0, A, B}
  float2 qab[fBQ];   // per query: pass iff product >= a * row value + b
};

template <typename XT>
struct FilterPre {  // one K chunk of X rows in flight
  i32x4 x[XPiece<XT>::P];
};
struct FilterPreQ {  // one K chunk of the (L2-resident) query tile
  i32x4 q[fQP];
};

// Buffer loads: a per-tile descriptor (its size clips rows past n to zero) and
// 32-bit per-lane offsets, the chunk offset in the scalar operand.
struct FilterAddr {
  __amdgpu_buffer_rsrc_t xr, qr;
  int d, dq;
  uint32_t xs, qs;  // byte strides between a thread's consecutive X / Q pieces
  uint32_t qb;      // byte stride between blocks of 32 query components
};

// A thread's offsets, derived once per tile from opaque(tid) (so they are not
// hoisted and kept live across the epilogue); a piece / K step / buffer then
// adds a wave-uniform or compile-time constant: no per-use address math in
// the K loop (v_mul_lo_u32 is quarter rate).
constexpr uint32_t kXB = sizeof(_Float16) * fBM * fLds;  // one LDS X buffer, bytes
constexpr uint32_t kQB = sizeof(_Float16) * fBQ * fLds;  // one LDS Q buffer, bytes
constexpr uint32_t kQOff = 2 * kXB;                      // FilterShared::qs
static_assert(__builtin_offsetof(FilterShared, qs) == kQOff, "LDS layout");
struct FilterOff {
  uint32_t xg, qg;  // global byte offsets of piece 0 (X within the tile, Q within the query tile)
  uint32_t xw, qw;  // LDS byte addresses of the stores of piece 0 (buffer 0)
  uint32_t xr, qr;  // LDS byte addresses of this lane's fragment reads (buffer 0)
  int kc;           // element offset of this lane's piece within a K chunk
};

template <typename XT>
__device__ __forceinline__ FilterOff filter_offsets(unsigned t, const FilterAddr& ad) {
  using X = XPiece<XT>;
  FilterOff o;
  o.kc = (int)(t % X::C) * X::E;
  o.xg = ((t / X::C) * (unsigned)ad.d + (t % X::C) * X::E) * (unsigned)sizeof(XT);
  // query piece p = t % fQC of a chunk: block p / 4, 16 B p % 4 of the query's 64
  o.qg = (t / fQC) * 64 + (t % fQC) % 4 * 16 + (t % fQC) / 4 * ad.qb;
  o.xw = ((t / X::C) * fLds + (t % X::C) * X::E) * 2;
  o.qw = kQOff + ((t / fQC) * fLds + (t % fQC) * 8) * 2;
  const unsigned lane = t & 63, wid = t >> 6;
  const unsigned rg = wid % fRG, qg = wid / fRG, h = lane >> 5, l32 = lane & 31;
  o.xr = ((rg * 64 + l32) * fLds + 8 * h) * 2;
  o.qr = kQOff + ((qg * fQT * 32 + l32) * fLds + 8 * h) * 2;
  return o;
}

template <typename T>
__device__ __forceinline__ T& lds_at(unsigned char* smem, uint32_t off) {
  return *reinterpret_cast<T*>(smem + off);
}

__device__ __forceinline__ void filter_load_q(FilterPreQ& p, const FilterAddr& ad,
                                              const FilterOff& o, int c, int diag) {
#pragma unroll
  for (int i = 0; i < fQP; ++i) {
    if (diag & 8) {
      p.q[i] = i32x4(0);
      continue;
    }
    // chunks past the padded row: an offset beyond the buffer (zeros)
    const uint32_t off = c * fBK < ad.dq ? o.qg + i * ad.qs : 0x7fff0000u;
    p.q[i] = __builtin_bit_cast(
        i32x4, __builtin_amdgcn_raw_buffer_load_b128(ad.qr, off, c * (fBK / 32) * ad.qb, 0));
  }
}

template <typename XT>
__device__ __forceinline__ void filter_load(FilterPre<XT>& p, const FilterAddr& ad,
                                            const FilterOff& o, int c) {
  const int k0 = c * fBK;
  // past the row end: an offset beyond the buffer (reads zeros)
  const uint32_t base = k0 + o.kc < ad.d ? o.xg : 0x7fff0000u;
#pragma unroll
  for (int i = 0; i < XPiece<XT>::P; ++i)
    p.x[i] = __builtin_bit_cast(
        i32x4, __builtin_amdgcn_raw_buffer_load_b128(ad.xr, base + i * ad.xs,
                                                     k0 * (int)sizeof(XT), 2 /* nt */));
}

// Stage one chunk into LDS buffer BUF: f32 rows to fp16 (with their sums of
// squares, as float pairs so the packed fma reads the loaded registers
// directly, and the max |x| for the fp16-overflow test), fp16 rows as they
// are (sums of squares of the exact f32 values; an fp16 row cannot overflow,
// an infinity or NaN shows in the sum), the query pieces as they are.
// IMG: the rows are the fp16 filter image of an f32 corpus (fx_filter_image);
// their row values come from FilterArgs::rowinfo instead.
template <typename XT, int BUF, bool IMG>
__device__ __forceinline__ void filter_store(const FilterPre<XT>& p, const FilterPreQ& pq,
                                             unsigned char* smem, const FilterOff& o,
                                             f32x2 (&sq)[XPiece<XT>::P],
                                             float (&mx)[XPiece<XT>::P]) {
  using X = XPiece<XT>;
#pragma unroll
  for (int i = 0; i < X::P; ++i) {
    const uint32_t at = o.xw + BUF * kXB + i * (fThreads / X::C) * fLds * 2;
    if constexpr (sizeof(XT) == 4) {
      const f32x4 v = __builtin_bit_cast(f32x4, p.x[i]);
      lds_at<f16x4>(smem, at) = __builtin_convertvector(v, f16x4);
      const f32x2 lo = {v[0], v[1]}, hi = {v[2], v[3]};
      sq[i] = __builtin_elementwise_fma(lo, lo, sq[i]);
      sq[i] = __builtin_elementwise_fma(hi, hi, sq[i]);
      mx[i] = fmaxf(mx[i],
                    fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    } else {
      lds_at<i32x4>(smem, at) = p.x[i];
      if constexpr (!IMG) {
        const f16x8 h = __builtin_bit_cast(f16x8, p.x[i]);
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const f32x2 v = {(float)h[e], (float)h[e + 1]};
          sq[i] = __builtin_elementwise_fma(v, v, sq[i]);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < fQP; ++i)
    lds_at<i32x4>(smem, o.qw + BUF * kQB + i * (fThreads / fQC) * fLds * 2) = pq.q[i];
}

// Hide a value from loop-invariant code motion: addresses derived from it are
// recomputed (a few VALU ops) where they are used instead of being hoisted out
// of the chunk loop and kept live (or spilled) across it.
__device__ __forceinline__ unsigned opaque(unsigned v) {
  asm volatile("" : "+v"(v));
  return v;
}

template <int BUF>
__device__ __forceinline__ void filter_compute(f32x16 (&acc)[2][fQT], unsigned char* smem,
                                               const FilterOff& o) {
#pragma unroll
  for (int s = 0; s < fBK / 16; ++s) {
    f16x8 av[2], bv[fQT];
#pragma unroll
    for (int t = 0; t < 2; ++t)
      av[t] = lds_at<f16x8>(smem, o.xr + BUF * kXB + (t * 32 * fLds + 16 * s) * 2);
#pragma unroll
    for (int u = 0; u < fQT; ++u)
      bv[u] = lds_at<f16x8>(smem, o.qr + BUF * kQB + (u * 32 * fLds + 16 * s) * 2);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < fQT; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[t], bv[u], acc[t][u], 0, 0, 0);
  }
}

// Calls f(integral_constant<int, I>) for I = 0 .. N-1 (indices stay static)
template <int N, typename F, int I = 0>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, F, I + 1>(static_cast<F&&>(f));
  }
}

// static_for when STATIC, else a plain unrolled loop (the compiler's choice)
template <bool STATIC, int N, typename F>
__device__ __forceinline__ void unroll_for(F&& f) {
  if constexpr (STATIC) {
    static_for<N>(static_cast<F&&>(f));
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) f(i);
  }
}

// Per-query constants of the pass test (once per block).  The test lb <= T
// is linear in the product x for a fixed row, so it is precomputed as
// x >= a * rv + b with rv the row's value (cosine: max(|x|, 1e-12); IP: |x|;
// L2: |x|^2):
//   cos  lb = x c1 / rv + 0.5 - A - B / rv,  c1 = -0.5 / (scale |q|) < 0
//        -> x >= ((T - 0.5 + A) rv + B) / c1
//   IP   lb = -x / scale - A rv - B           -> x >= (-T - B - A rv) scale
//   L2   lb^2 = s2 - 2 x / scale - A s2 - B,  s2 = rv + |q|^2, against
//        T^2 (1 + 2^-20) -> x >= ((1 - A) s2 - B - T^2) scale / 2
// The roundings of this rearrangement are far inside the bound's slack.
// T = NaN (no threshold yet) or a forced query: everything passes
// (a = 0, b = -inf); padding queries: nothing (b = +inf).  qtab keeps
// {c1, c0, A, B} for the exact bounds of appended pairs.
template <int METRIC>
__device__ __forceinline__ void filter_query_table(const FilterArgs& a, int64_t q0, f32x4* qtab,
                                                   float2* qab, int tid, int nthreads) {
  for (int i = tid; i < fBQ; i += nthreads) {
    const int64_t gq = q0 + i;
    f32x4 c = f32x4(0.f);
    float2 ab = {0.f, __builtin_inff()};
    if (gq < a.nq) {
      const f32x4 info = *reinterpret_cast<const f32x4*>(a.qinfo + gq * 4);
      float tf = key_float((uint32_t)(a.thr[gq] >> 32));
      const float qinv = info[0], qa = info[1], qA = info[2], qB = info[3];
      c[2] = qA;
      c[3] = qB;
      // the upper-bound test (ub_test): the same forms with the error terms
      // A, B negated, and T widened by 2^-14 relative (the rows that set T
      // pass again; extra passes only cost an append)
      const float sA = a.ub_test ? -qA : qA, sB = a.ub_test ? -qB : qB;
      if (a.ub_test) tf += fabsf(tf) * 6.103515625e-05f;
      if constexpr (METRIC == 0) {
        c[0] = -2.f * qinv;
        c[1] = qa;
        const float t2 = tf * tf * (1.f + 9.5367431640625e-07f);
        const float h = 0.5f / qinv;
        ab.x = (1.f - sA) * h;
        ab.y = ((1.f - sA) * qa - sB - t2) * h;
      } else if constexpr (METRIC == 1) {
        c[0] = -qinv;
        const float sc = 1.f / qinv;
        ab.x = -sA * sc;
        ab.y = (-tf - sB) * sc;
      } else {
        c[0] = -0.5f * qinv / qa;
        ab.x = (tf - 0.5f + sA) / c[0];
        ab.y = sB / c[0];
      }
      if (tf != tf || !(qA <= 3.4e38f)) ab = {0.f, -__builtin_inff()};
    }
    qtab[i] = c;
    qab[i] = ab;
  }
}

// Where local row lr of a 256-row tile sits in the epilogue's masks when a
// wave owns RT 32-row MFMA tiles: the word of its (32 RT-row group, lane
// half) and its bit there, j with lr = 32 RT rg + 4 h + roff(j)
// (filter_epilogue).
template <int RT>
__device__ __forceinline__ void filter_row_bit(int lr, int& word, int& bit) {
  const int w = lr % (32 * RT), w2 = lr & 31;
  word = (lr / (32 * RT)) * 2 + ((w2 >> 2) & 1);
  bit = (w >> 5) * 16 + (w2 >> 3) * 4 + (w2 & 3);
}

// Record one row's bound factor for the epilogue (rv NaN: forced through,
// ok false: skipped), the cosine term 1 / rv of its appends, and its flags
// (words zeroed at the tile start, ordered by the K loop's barriers).
template <int METRIC, int RT = 2>
__device__ __forceinline__ void filter_note_row(float* rinfo, float* rterm, uint32_t* flags,
                                                int lr, float rv, bool ok) {
  rinfo[lr] = ok ? rv : -1.f;
  if constexpr (METRIC == 2) rterm[lr] = 1.f / rv;
  int word, bit;
  filter_row_bit<RT>(lr, word, bit);
  if (!ok) atomicOr(&flags[16 + word], 1u << bit);
  else if (rv != rv) atomicOr(&flags[word], 1u << bit);
}

// Epilogue of one tile: pass test per (row, query) — an fma, a subtraction
// and a funnel shift that collects the sign of (product - threshold) (see
// filter_query_table; extra passes only cost a rescored candidate); the
// lane's passes over its 16 RT rows form a bit mask per query column, one
// atomic per (lane, column) reserves their slots.  Forced rows (flag words
// 0..15) always pass, skipped rows (16..31) never.
template <int METRIC, int QT, int RT = 2>
__device__ __forceinline__ void filter_epilogue(const f32x16 (&acc)[RT][QT], const float* rinfo,
                                                const float* rterm, const uint32_t* flags,
                                                const f32x4* qtab, const float2* qab,
                                                const FilterArgs& a, int64_t q0, int64_t r0,
                                                int rg, int qg, int h, int l32, int diag) {
    constexpr int NR = 16 * RT;  // rows per lane
    constexpr uint32_t kAll = NR == 32 ? ~0u : (1u << NR) - 1u;
    const int lr0 = rg * 32 * RT + 4 * h;
    const float* ri = rinfo + lr0;
    const uint32_t grow0 = (uint32_t)(a.row_base + r0 + lr0);
    // row j of the lane (acc register j & 15 of row tile j >> 4) sits at a
    // compile-time offset from ri: row values are re-read from LDS where used
    auto roff = [](int j) { return (j >> 4) * 32 + (j & 3) + 8 * ((j & 15) >> 2); };
    const uint32_t fmask = flags[rg * 2 + h], smask = flags[16 + rg * 2 + h];
    uint32_t pm[QT];
#pragma unroll
    for (int u = 0; u < QT; ++u) {
      const float2 ab = qab[qg * QT * 32 + u * 32 + l32];
      // fail bits: sign of RN(x - t) is set exactly when x < t (x, t finite;
      // RN never flips a sign, x == t gives +0); bit j enters last-in at
      // bit 0, so j runs down
      uint32_t fail = 0u;
#pragma unroll
      for (int j = NR - 1; j >= 0; --j) {
        const float t = fmaf(ab.x, ri[roff(j)], ab.y);
        fail = __builtin_amdgcn_alignbit(fail, __float_as_uint(acc[j >> 4][u][j & 15] - t), 31);
      }
      pm[u] = (diag & 1) ? 0u : ((~fail | fmask) & ~smask & kAll);
      if (q0 + qg * QT * 32 + u * 32 + l32 >= a.nq) pm[u] = 0u;
    }
    uint32_t any = 0u;
#pragma unroll
    for (int u = 0; u < QT; ++u) any |= pm[u];
    if (__ballot(any != 0u) == 0ull) return;
    uint32_t pos[QT];
#pragma unroll
    for (int u = 0; u < QT; ++u) {
      pos[u] = 0u;
      const int64_t gq = q0 + qg * QT * 32 + u * 32 + l32;
      if (pm[u] != 0u) {
        if ((diag & 32) && a.cand_ub != nullptr)  // profiling only (final phase): no atomic
          pos[u] = (uint32_t)l32 * 64u;
        else
          pos[u] = atomicAdd(&a.count[gq * kCountStride], (uint32_t)__popc(pm[u]));
      }
    }
#pragma unroll
    for (int u = 0; u < QT; ++u) {
      if (__ballot(pm[u] != 0u) == 0ull) continue;
      const int qi = qg * QT * 32 + u * 32 + l32;
      const int64_t gq = q0 + qi;
      const f32x4 qc = qtab[qi];
      const float qc1 = qc[0], qc0 = qc[1], qA = qc[2], qB = qc[3];
      const bool fq = !(qA <= 3.4e38f);
      uint32_t p = pos[u];
      // rows in groups of 4: a group no lane of the wave appends from is
      // skipped with one wave-uniform branch (a few appends per wave and tile)
#pragma unroll
      for (int g = 0; g < NR / 4; ++g) {
        if (__ballot(((pm[u] >> (4 * g)) & 0xfu) != 0u) == 0ull) continue;
#pragma unroll
      for (int j = 4 * g; j < 4 * g + 4; ++j) {
        if (!((pm[u] >> j) & 1u)) continue;
        const float rv = ri[roff(j)];
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
          const float rt = rterm[lr0 + roff(j)];
          const float dist = fmaf(x * rt, qc1, 0.5f);
          const float e = fmaf(qB, rt, qA);
          lb = dist - e;
          ub = dist + e;
        }
        if (fq || rv != rv) {  // forced: below / above every key
          lb = -__builtin_inff();
          ub = __builtin_nanf("");
        }
        if (p < (uint32_t)a.cap && !((diag & 64) && a.cand_ub != nullptr)) {  // (64: profiling)
          const uint32_t grow = grow0 + (uint32_t)roff(j);
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

// filter_epilogue with the appends staged in LDS: they go to a per-(workgroup, query) LDS segment of SEG
// entries {lb key, ub key, row} (slot from an LDS atomic: no global atomic
// and no global store on the tile boundary), flushed at the kernel's end
// (filter_flush_segments); entries past SEG take a global slot as before.
template <int METRIC, int QT, int RT, int SEG>
__device__ __forceinline__ void filter_epilogue_seg(const f32x16 (&acc)[RT][QT], const float* rinfo,
                                                const float* rterm, const uint32_t* flags,
                                                const f32x4* qtab, const float2* qab,
                                                const FilterArgs& a, int64_t q0, int64_t r0,
                                                int rg, int qg, int h, int l32, int diag,
                                                uint32_t* seg) {
    constexpr int NR = 16 * RT;  // rows per lane
    constexpr uint32_t kAll = NR == 32 ? ~0u : (1u << NR) - 1u;
    const int lr0 = rg * 32 * RT + 4 * h;
    const float* ri = rinfo + lr0;
    const uint32_t grow0 = (uint32_t)(a.row_base + r0 + lr0);
    // row j of the lane (acc register j & 15 of row tile j >> 4) sits at a
    // compile-time offset from ri: row values are re-read from LDS where used
    auto roff = [](int j) { return (j >> 4) * 32 + (j & 3) + 8 * ((j & 15) >> 2); };
    const uint32_t fmask = flags[rg * 2 + h], smask = flags[16 + rg * 2 + h];
    uint32_t pm[QT];
#pragma unroll
    for (int u = 0; u < QT; ++u) {
      const float2 ab = qab[qg * QT * 32 + u * 32 + l32];
      // fail bits: sign of RN(x - t) is set exactly when x < t (x, t finite;
      // RN never flips a sign, x == t gives +0); bit j enters last-in at
      // bit 0, so j runs down
      uint32_t fail = 0u;
#pragma unroll
      for (int j = NR - 1; j >= 0; --j) {
        const float t = fmaf(ab.x, ri[roff(j)], ab.y);
        fail = __builtin_amdgcn_alignbit(fail, __float_as_uint(acc[j >> 4][u][j & 15] - t), 31);
      }
      pm[u] = (diag & 1) ? 0u : ((~fail | fmask) & ~smask & kAll);
      if (q0 + qg * QT * 32 + u * 32 + l32 >= a.nq) pm[u] = 0u;
    }
    uint32_t any = 0u;
#pragma unroll
    for (int u = 0; u < QT; ++u) any |= pm[u];
    if (__ballot(any != 0u) == 0ull) return;
    uint32_t pos[QT];
#pragma unroll
    for (int u = 0; u < QT; ++u) {
      pos[u] = 0u;
      const int64_t gq = q0 + qg * QT * 32 + u * 32 + l32;
      if (pm[u] != 0u) {
        if constexpr (SEG > 0)  // LDS counter of the query (seg[0 .. fBQ))
          pos[u] = atomicAdd(&seg[qg * QT * 32 + u * 32 + l32], (uint32_t)__popc(pm[u]));
        else if ((diag & 32) && a.cand_ub != nullptr)  // profiling only (final phase): no atomic
          pos[u] = (uint32_t)l32 * 64u;
        else
          pos[u] = atomicAdd(&a.count[gq * kCountStride], (uint32_t)__popc(pm[u]));
      }
    }
    unroll_for<(SEG > 0), QT>([&](auto uc) {
      const int u = uc;
      if (__ballot(pm[u] != 0u) == 0ull) return;
      const int qi = qg * QT * 32 + u * 32 + l32;
      const int64_t gq = q0 + qi;
      const f32x4 qc = qtab[qi];
      const float qc1 = qc[0], qc0 = qc[1], qA = qc[2], qB = qc[3];
      const bool fq = !(qA <= 3.4e38f);
      uint32_t p = pos[u];
      uint32_t gp = ~0u;
      // rows in groups of 4: a group no lane of the wave appends from is
      // skipped with one wave-uniform branch (a few appends per wave and tile)
      unroll_for<(SEG > 0), NR / 4>([&](auto gc) {
        const int g = gc;
        if (__ballot(((pm[u] >> (4 * g)) & 0xfu) != 0u) == 0ull) return;
      unroll_for<(SEG > 0), 4>([&](auto jc) {
        const int j = 4 * g + (int)jc;
        if (!((pm[u] >> j) & 1u)) return;
        const float rv = ri[roff(j)];
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
          const float rt = rterm[lr0 + roff(j)];
          const float dist = fmaf(x * rt, qc1, 0.5f);
          const float e = fmaf(qB, rt, qA);
          lb = dist - e;
          ub = dist + e;
        }
        if (fq || rv != rv) {  // forced: below / above every key
          lb = -__builtin_inff();
          ub = __builtin_nanf("");
        }
        if constexpr (SEG > 0) {
          const uint32_t grow = grow0 + (uint32_t)roff(j);
          if (p < (uint32_t)SEG) {
            uint32_t* e = seg + fBQ + 3 * (qi * SEG + p);
            e[0] = order_key(lb);
            e[1] = order_key(ub);
            e[2] = grow;
          } else {  // rare: past the segment, global slots for the lane's remaining passes
            if (gp == ~0u) gp = atomicAdd(&a.count[gq * kCountStride], (uint32_t)__popc(pm[u] >> j));
            if (gp < (uint32_t)a.cap) {
              const size_t slot = (size_t)gq * a.cap + gp;
              if (a.cand_ub != nullptr) {
                a.cand[slot] = make_comp(lb, grow);
                a.cand_ub[slot] = make_comp(ub, grow);
              } else {
                a.cand[slot] = make_comp(ub, grow);
              }
            }
            ++gp;
          }
        } else
        if (p < (uint32_t)a.cap && !((diag & 64) && a.cand_ub != nullptr)) {  // (64: profiling)
          const uint32_t grow = grow0 + (uint32_t)roff(j);
          const size_t slot = (size_t)gq * a.cap + p;
          if (a.cand_ub != nullptr) {
            a.cand[slot] = make_comp(lb, grow);
            a.cand_ub[slot] = make_comp(ub, grow);
          } else {
            a.cand[slot] = make_comp(ub, grow);
          }
        }
        ++p;
      });
      });
    });
}

// The tile loop of filter_kernel.  SF (store first): the wave stores chunk
// c + 1 and issues its loads before it multiplies chunk c, instead of after.
// Both orders are legal inside one barrier interval (the two touch different
// LDS buffers); with FX_FILTER_SPLIT the second half of the workgroup (waves
// fWaves/2.., each the SIMD partner of a first-half wave) takes the other
// order, so one wave of a SIMD issues its MFMAs while its partner converts,
// stores and loads, instead of both doing each phase together.
template <typename XT, int METRIC, bool IMG, bool SF, typename Diag>
__device__ __forceinline__ void filter_tiles(const FilterArgs& a, unsigned char* smem, int tid,
                                             Diag diag) {
  using X = XPiece<XT>;
  FilterShared* sh = reinterpret_cast<FilterShared*>(smem);
  const int lane = tid & 63, wid = tid >> 6;
  const int rg = wid % fRG, qg = wid / fRG;  // 64-row group, fQT*32-query group
  const int h = lane >> 5, l32 = lane & 31;
  const int64_t q0 = (int64_t)blockIdx.y * fBQ;
  const int nch = (a.d + fBK - 1) / fBK;

  // the buffer descriptor of the X rows of the tile at row r0 (rows past n,
  // or a tile past the end, read as zeros)
  auto x_rsrc = [&](int64_t r0) {
    int64_t rows = a.n - r0 < fBM ? a.n - r0 : fBM;
    if (rows < 0) rows = 0;
    const XT* xb = reinterpret_cast<const XT*>(a.X) + (rows > 0 ? r0 : 0) * (int64_t)a.d;
    const uint64_t xp = reinterpret_cast<uint64_t>(xb);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)xp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(xp >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)(rows * a.d * (int64_t)sizeof(XT)));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                             nb, 0x00020000);
  };
  auto tile_r0 = [&](int64_t ti) { return (a.tile_start + ti * a.tile_stride) * fBM; };
  FilterAddr ad;
  {
    const uint16_t* qb = a.Qh + q0 * 32;
    const uint64_t qp = reinterpret_cast<uint64_t>(qb);
    const uint32_t qlo = __builtin_amdgcn_readfirstlane((uint32_t)qp);
    const uint32_t qhi = __builtin_amdgcn_readfirstlane((uint32_t)(qp >> 32));
    const int qnb = __builtin_amdgcn_readfirstlane(
        (int)(((int64_t)(a.dq / 32 - 1) * a.qstride + fBQ) * 64));
    ad.qr = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)qhi << 32) | qlo), 0, qnb, 0x00020000);
    ad.d = a.d;
    ad.xs = (uint32_t)(fThreads / X::C) * (uint32_t)a.d * (uint32_t)sizeof(XT);
    ad.qs = (uint32_t)(fThreads / fQC) * 64u;
    ad.qb = (uint32_t)a.qstride * 64u;
    ad.dq = a.dq;
  }

  // Two register stages: chunks c + 2 and c + 3 of X are in flight while
  // chunk c is multiplied (stage j % 2 holds chunk j), the query tile one
  // chunk ahead.  Loads are issued unconditionally (chunks past the row end
  // read as zeros through the descriptor bounds): a load under a branch
  // makes the compiler wait for it where the branch joins.  With kXpf a
  // tile's first two X chunks and first query chunk are issued before the
  // previous tile's epilogue (the stages are free by then), so they stream
  // in while it runs.
  FilterPre<XT> pf[2];
  FilterPreQ pq;
  int64_t ti = blockIdx.x;
  if constexpr (kXpf) {
    ad.xr = x_rsrc(tile_r0(ti));
    const FilterOff o = filter_offsets<XT>(opaque(tid), ad);
    filter_load_q(pq, ad, o, 0, diag);
    filter_load(pf[0], ad, o, 0);
    filter_load(pf[1], ad, o, 1);
  }
  int par = 0;  // tile parity: which rflags words this tile's epilogue reads
  for (; ti < a.num_tiles; ti += gridDim.x, par ^= 1) {
    const int64_t r0 = tile_r0(ti);
    // (last read by the epilogue two tiles back: every wave has passed the
    // previous tile's barriers since)
    if (tid < kRowFlagWords) sh->rflags[par][tid] = 0u;

    f32x16 acc[2][fQT];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < fQT; ++u) acc[t][u] = f32x16(0.f);
    f32x2 sq[X::P];
    float mx[X::P];
#pragma unroll
    for (int i = 0; i < X::P; ++i) {
      sq[i] = f32x2(0.f);
      mx[i] = 0.f;
    }

    ad.xr = x_rsrc(r0);
    const FilterOff o = filter_offsets<XT>(opaque(tid), ad);
    if constexpr (!kXpf) {
      filter_load_q(pq, ad, o, 0, diag);
      filter_load(pf[0], ad, o, 0);
      filter_load(pf[1], ad, o, 1);
    }
    filter_store<XT, 0, IMG>(pf[0], pq, smem, o, sq, mx);
    // Q one chunk ahead, issued before the X load of the same step: vmcnt
    // retires loads in issue order, so waiting for Q(c + 1) at step c waits
    // for X(c + 1) (needed there anyway) and nothing issued later.
    filter_load_q(pq, ad, o, 1, diag);
    filter_load(pf[0], ad, o, 2);
    __syncthreads();
    // One K step: multiply chunk c (LDS buffer c & 1 = B), store chunk c + 1
    // from its stage p into the other buffer, refill p with chunk c + 3.  The
    // main loop runs only full steps, with no branch inside (a conditional
    // store or load makes the waitcnt pass merge pending-load states at the
    // join and wait for every load in flight, draining the stream).
    auto step = [&](int c, FilterPre<XT>& p, auto buf) {
      constexpr int B = decltype(buf)::value;
      if constexpr (!SF) {
        if (!(diag & 4)) filter_compute<B>(acc, smem, o);
      }
      if (!(diag & 16)) filter_store<XT, B ^ 1, IMG>(p, pq, smem, o, sq, mx);
      filter_load_q(pq, ad, o, c + 2, diag);
      filter_load(p, ad, o, c + 3);
      if constexpr (SF) {
        if (!(diag & 4)) filter_compute<B>(acc, smem, o);
      }
      __syncthreads();
    };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    int c = 0;
    for (; c + 2 < nch; c += 2) {
      step(c, pf[1], B0{});
      step(c + 1, pf[0], B1{});
    }
    // the last one or two chunks (c is even: chunk c sits in buffer 0, chunk
    // c + 1, if any, in stage 1); one-sided branches only, so the
    // accumulators need no copies at a join
    const bool two = c + 1 < nch;
    if (two && !(diag & 16)) filter_store<XT, 1, IMG>(pf[1], pq, smem, o, sq, mx);
    __syncthreads();
    // kXpf: the rows' image sums and mask words for the epilogue, issued
    // before the last chunks' MFMAs and the next tile's loads, so they are in
    // when it starts without waiting for those
    float img_sq[X::P];
    uint32_t mword[X::P];
    if constexpr (kXpf) {
#pragma unroll
      for (int i = 0; i < X::P; ++i) {
        const int lr = (i * fThreads + tid) / X::C;
        const int64_t row = r0 + lr < a.n ? r0 + lr : a.n - 1;
        if constexpr (IMG) img_sq[i] = a.rowinfo[row];
        mword[i] = a.mask != nullptr ? a.mask[row >> 5] : ~0u;
      }
    }
    if (!(diag & 4)) filter_compute<0>(acc, smem, o);
    if (two && !(diag & 4)) filter_compute<1>(acc, smem, o);
    if constexpr (kXpf) {  // the next tile's first chunks (past the end: an empty descriptor)
      const int64_t tn = ti + gridDim.x;
      ad.xr = x_rsrc(tn < a.num_tiles ? tile_r0(tn) : a.n);
      const FilterOff on = filter_offsets<XT>(opaque(tid), ad);
      filter_load_q(pq, ad, on, 0, diag);
      filter_load(pf[0], ad, on, 0);
      filter_load(pf[1], ad, on, 1);
    }

    // per-row value rv from |x|^2 (the fRowLanes lanes of a row hold partials;
    // IMG: the f32 row's, precomputed): cosine max(|x|, 1e-12), IP |x|, L2
    // |x|^2; NaN = forced through (fp16 overflow: a component >= 65520;
    // non-finite); -1 = skipped (past n or masked out)
    float sqs[X::P];
#pragma unroll
    for (int i = 0; i < X::P; ++i) {
      sqs[i] = sq[i][0] + sq[i][1];
      if constexpr (!IMG) {
#pragma unroll
        for (int m = 1; m < X::C; m <<= 1) {
          sqs[i] += __shfl_xor(sqs[i], m);
          mx[i] = fmaxf(mx[i], __shfl_xor(mx[i], m));
        }
      }
    }
#pragma unroll
    for (int i = 0; i < X::P; ++i) {
      if (tid % X::C == 0) {
        const int lr = (i * fThreads + tid) / X::C;
        const int64_t row = r0 + lr;
        bool ok = row < a.n;
        if constexpr (kXpf) {
          if constexpr (IMG) sqs[i] = ok ? img_sq[i] : 0.f;
          if (ok) ok = (mword[i] >> (row & 31)) & 1u;
        } else {
          if constexpr (IMG) sqs[i] = ok ? a.rowinfo[row] : 0.f;
          if (ok && a.mask != nullptr) ok = (a.mask[row >> 5] >> (row & 31)) & 1u;
        }
        float rv;
        if constexpr (METRIC == 0) {
          rv = sqs[i];
        } else if constexpr (METRIC == 1) {
          rv = sqrtf(sqs[i]);
        } else {
          rv = fmaxf(sqrtf(sqs[i]), 1e-12f);
        }
        if (!(sqs[i] <= 3.4e38f) || mx[i] >= 65520.f) rv = __builtin_nanf("");
        filter_note_row<METRIC>(sh->rinfo, sh->rterm, sh->rflags[par], lr, rv, ok);
      }
    }
    __syncthreads();

    // ---- epilogue: [lb, ub] per (row, query), threshold test, append
    if (diag & 2) {
      if (acc[0][0][0] == 1.2345f && acc[1][fQT - 1][5] == 2.f) a.count[0] = 7;
      continue;
    }

    filter_epilogue<METRIC, fQT>(acc, sh->rinfo, sh->rterm, sh->rflags[par], sh->qtab, sh->qab, a,
                                 q0, r0, rg, qg, h, l32, diag);
  }
}

// Write a workgroup's LDS append segments (filter_epilogue_seg) to the
// candidate buffer: one global atomic per query reserves the slots.  seg =
// [fBQ counters][fBQ x SEG entries {lb key, ub key, row}]; called by every
// thread after the last tile (ends with the counters reused as bases).
// segcap: entries per query (SEG, or more when the slice has fewer live
// queries: i8_epilogue's segcap), fBQ * SEG entries in all.
template <int SEG, int NT = fThreads>
__device__ __forceinline__ void filter_flush_segments(uint32_t* seg, uint32_t* base,
                                                      const FilterArgs& a, int64_t q0, int tid,
                                                      int segcap = SEG) {
  __syncthreads();
  for (int q = tid; q < fBQ; q += NT) {
    const uint32_t n = seg[q] < (uint32_t)segcap ? seg[q] : (uint32_t)segcap;
    seg[q] = n;
    base[q] = n != 0u && q0 + q < a.nq ? atomicAdd(&a.count[(q0 + q) * kCountStride], n) : 0u;
  }
  __syncthreads();
  for (int i = tid; i < fBQ * SEG; i += NT) {
    const int q = i / segcap, j = i % segcap;
    if (q >= fBQ || (uint32_t)j >= seg[q]) continue;
    const uint32_t p = base[q] + (uint32_t)j;
    if (p >= (uint32_t)a.cap) continue;
    const uint32_t* e = seg + fBQ + 3 * i;
    const size_t slot = (size_t)(q0 + q) * a.cap + p;
    if (a.cand_ub != nullptr) {
      a.cand[slot] = ((uint64_t)e[0] << 32) | e[2];
      a.cand_ub[slot] = ((uint64_t)e[1] << 32) | e[2];
    } else {
      a.cand[slot] = ((uint64_t)e[1] << 32) | e[2];
    }
  }
}

// ------------------------------------------------------ tiled filter image
#ifndef FX_FILTER_IMG2  // compiled into the 64-query and the 32-wide-K 256-query builds
                        // (the 64-wide-K h256 build measured 7 % slower on it)
#define FX_FILTER_IMG2 (FX_FILTER_BQ <= 128 || FX_FILTER_BK == 32)
#endif
#ifndef FX_I2_SEG  // LDS append segment per query (0: a global atomic per lane and query);
                   // 64-query tiles only: 16 entries in the 256-query build (the most
                   // its LDS holds) measured 3.5 % slower
#define FX_I2_SEG (FX_FILTER_BQ >= 256 ? 0 : 32)
#endif
//
// The fp16 image of an f32 corpus in MFMA fragment order (FX_IMAGE_TILED,
// default on), [ceil(n / 32) row tiles][ceil(d / 16) k-steps][64 lanes][8
// halves]: lane l holds row 32 t + l % 32, components 16 s + 8 (l / 32) ..
// + 7, i.e. one v_mfma_f32_32x32x16_f16 A operand, one contiguous KB per wave
// load.  Each of the 8 waves owns one 32-row tile of the 256-row tile against
// all the queries and loads its A fragments straight into registers (two
// chunks ahead); only the query tile goes through LDS.
struct Img2Shared {
  _Float16 qs[2][fBQ * fLds];
  float rinfo[fBM];
  float rterm[fBM];
  uint32_t rflags[2][kRowFlagWords];
  f32x4 qtab[fBQ];
  float2 qab[fBQ];
#if FX_I2_SEG > 0
  uint32_t seg[fBQ + 3 * fBQ * FX_I2_SEG];  // counters, then entries (filter_epilogue_seg)
  uint32_t segbase[fBQ];
#endif
};
static_assert(sizeof(Img2Shared) <= 160 * 1024, "filter_img2_kernel: LDS over 160 KB");
constexpr int kI2QT = fBQ / 32;  // query tiles per wave (every query)
constexpr int kI2KS = fBK / 16;  // k-steps per chunk
static_assert(fWaves * 32 == fBM, "tiled image: one 32-row tile per wave");

template <int METRIC>
__global__ void __launch_bounds__(fThreads, fWaves / 4) filter_img2_kernel(FilterArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  Img2Shared* sh = reinterpret_cast<Img2Shared*>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, l32 = lane & 31;
  const int64_t q0 = (int64_t)blockIdx.y * fBQ;
  const int nch = (a.d + fBK - 1) / fBK;
  const int ksteps = (a.d + 15) / 16;
  const int64_t ntile32 = (a.n + 31) / 32;
#ifdef FX_DIAG_BUILD
  const int diag = a.diag;
#else
  constexpr int diag = 0;
#endif
  filter_query_table<METRIC>(a, q0, sh->qtab, sh->qab, tid, fThreads);
#if FX_I2_SEG > 0
  for (int q = tid; q < fBQ; q += fThreads) sh->seg[q] = 0u;  // (ordered by the tile barriers)
#endif

  FilterAddr ad;  // the query tile (as filter_tiles)
  {
    const uint16_t* qb = a.Qh + q0 * 32;
    const uint64_t qp = reinterpret_cast<uint64_t>(qb);
    const uint32_t qlo = __builtin_amdgcn_readfirstlane((uint32_t)qp);
    const uint32_t qhi = __builtin_amdgcn_readfirstlane((uint32_t)(qp >> 32));
    const int qnb = __builtin_amdgcn_readfirstlane(
        (int)(((int64_t)(a.dq / 32 - 1) * a.qstride + fBQ) * 64));
    ad.qr = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)qhi << 32) | qlo), 0, qnb, 0x00020000);
    ad.d = a.d;
    ad.xs = 0;
    ad.qs = (uint32_t)(fThreads / fQC) * 64u;
    ad.qb = (uint32_t)a.qstride * 64u;
    ad.dq = a.dq;
  }
  FilterOff o = {};
  {
    const unsigned t = opaque(tid);
    o.qg = (t / fQC) * 64 + (t % fQC) % 4 * 16 + (t % fQC) / 4 * ad.qb;
  }
  const uint32_t qw = ((tid / fQC) * fLds + (tid % fQC) * 8) * 2;  // this thread's Q stores
  const uint32_t qr = (l32 * fLds + 8 * h) * 2;                    // this lane's B fragments

  auto store_q = [&](const FilterPreQ& pq, auto buf) {
    constexpr int B = decltype(buf)::value;
#pragma unroll
    for (int i = 0; i < fQP; ++i)
      lds_at<i32x4>(smem, B * kQB + qw + i * (fThreads / fQC) * fLds * 2) = pq.q[i];
  };
  typedef f16x8 XA[kI2KS];
  int par = 0;
  for (int64_t ti = blockIdx.x; ti < a.num_tiles; ti += gridDim.x, par ^= 1) {
    const int64_t r0 = (a.tile_start + ti * a.tile_stride) * fBM;
    if (tid < kRowFlagWords) sh->rflags[par][tid] = 0u;
#ifndef FX_I2_RPF
#define FX_I2_RPF 1
#endif
    // this thread's row sum, loaded before the stream (not a dependent HBM
    // load between the last MFMA and the epilogue's barrier)
    float rsum = 0.f;
    if (FX_I2_RPF && tid < fBM && r0 + tid < a.n) rsum = a.rowinfo[r0 + tid];
    // this wave's 32-row tile: its k-steps, one KB each (a tile past the end
    // reads zeros through the descriptor size)
    __amdgpu_buffer_rsrc_t xr;
    {
      const int64_t t32 = r0 / 32 + wid;
      const int64_t live = t32 < ntile32 ? 1 : 0;
      const unsigned char* base = reinterpret_cast<const unsigned char*>(a.X) +
                                  (live ? t32 : 0) * (int64_t)ksteps * 1024;
      const uint64_t xp = reinterpret_cast<uint64_t>(base);
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)xp);
      const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(xp >> 32));
      const int nb = __builtin_amdgcn_readfirstlane((int)(live * ksteps * 1024));
      xr = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                             nb, 0x00020000);
    }
    const uint32_t xl = (uint32_t)opaque(lane) * 16u;
    auto load_x = [&](XA& xa, int c) {
#pragma unroll
      for (int s = 0; s < kI2KS; ++s) {
        const int ks = c * kI2KS + s;  // wave-uniform: past the row end reads zeros
        const uint32_t off = ks < ksteps ? xl : 0x7fff0000u;
        xa[s] = __builtin_bit_cast(
            f16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, off, ks * 1024, 2 /* nt */));
      }
    };
    f32x16 acc[1][kI2QT];
#pragma unroll
    for (int u = 0; u < kI2QT; ++u) acc[0][u] = f32x16(0.f);
    auto compute = [&](const XA& xa, auto buf) {
      constexpr int B = decltype(buf)::value;
      if (diag & 4) {  // (diagnostics: no MFMA; the row loads stay live)
        if (xa[0][0] == (_Float16)1.2345f && xa[kI2KS - 1][7] == (_Float16)2.f) a.count[0] = 7;
        return;
      }
#pragma unroll
      for (int s = 0; s < kI2KS; ++s) {
#pragma unroll
        for (int u = 0; u < kI2QT; ++u) {
          const f16x8 bv = lds_at<f16x8>(smem, B * kQB + qr + (u * 32 * fLds + 16 * s) * 2);
          acc[0][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa[s], bv, acc[0][u], 0, 0, 0);
        }
      }
    };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    FilterPreQ pq;
    XA xa0, xa1;
    filter_load_q(pq, ad, o, 0, diag);
    load_x(xa0, 0);
    load_x(xa1, 1);
    store_q(pq, B0{});
    filter_load_q(pq, ad, o, 1, diag);
    __syncthreads();
    // step c: multiply chunk c (registers xa[c & 1], query buffer c & 1),
    // store query chunk c + 1, load query chunk c + 2 and rows chunk c + 2
    auto step = [&](int c, XA& xa, auto buf) {
      constexpr int B = decltype(buf)::value;
      compute(xa, buf);
      store_q(pq, std::integral_constant<int, B ^ 1>{});
      filter_load_q(pq, ad, o, c + 2, diag);
      load_x(xa, c + 2);
      __syncthreads();
    };
    int c = 0;
    for (; c + 2 < nch; c += 2) {
      step(c, xa0, B0{});
      step(c + 1, xa1, B1{});
    }
    const bool two = c + 1 < nch;
    if (two) store_q(pq, B1{});
    __syncthreads();
    compute(xa0, B0{});
    if (two) compute(xa1, B1{});

    if (tid < fBM) {  // one thread per row: bound factor, flags
      const int lr = tid;
      const int64_t row = r0 + lr;
      bool ok = row < a.n;
      const float s = ok ? (FX_I2_RPF ? rsum : a.rowinfo[row]) : 0.f;
      if (ok && a.mask != nullptr) ok = (a.mask[row >> 5] >> (row & 31)) & 1u;
      float rv;
      if constexpr (METRIC == 0) {
        rv = s;
      } else if constexpr (METRIC == 1) {
        rv = sqrtf(s);
      } else {
        rv = fmaxf(sqrtf(s), 1e-12f);
      }
      if (!(s <= 3.4e38f)) rv = __builtin_nanf("");
      filter_note_row<METRIC, 1>(sh->rinfo, sh->rterm, sh->rflags[par], lr, rv, ok);
    }
    __syncthreads();
    if (diag & 2) {
      if (acc[0][0][0] == 1.2345f) a.count[0] = 7;
      continue;
    }
#if FX_I2_SEG > 0
    filter_epilogue_seg<METRIC, kI2QT, 1, FX_I2_SEG>(acc, sh->rinfo, sh->rterm, sh->rflags[par],
                                                 sh->qtab, sh->qab, a, q0, r0, wid, 0, h, l32,
                                                 diag, sh->seg);
#else
    filter_epilogue<METRIC, kI2QT, 1>(acc, sh->rinfo, sh->rterm, sh->rflags[par], sh->qtab,
                                      sh->qab, a, q0, r0, wid, 0, h, l32, diag);
#endif
  }
#if FX_I2_SEG > 0
  filter_flush_segments<FX_I2_SEG>(sh->seg, sh->segbase, a, q0, tid);
#endif
}

#if FX_FILTER_IMG2 && !FX_FILTER_IMG3
static int launch_img2(const FilterArgs& a, int metric, hipStream_t stream) {
  const size_t smem = sizeof(Img2Shared);
  const void* fn = metric == FX_METRIC_COS ? (const void*)filter_img2_kernel<2>
                   : metric == FX_METRIC_IP ? (const void*)filter_img2_kernel<1>
                                            : (const void*)filter_img2_kernel<0>;
  if (int rc = allow_lds(fn)) return rc;
  int cus = 0;
  int rc = device_cus(&cus);
  if (rc) return rc;
  const int64_t qtiles = (a.nq + fBQ - 1) / fBQ;
  int64_t bx = cus;
  if (bx > a.num_tiles) bx = a.num_tiles;
  for (int64_t y0 = 0; y0 < qtiles; y0 += 65535) {
    FilterArgs b = a;
    const int64_t yn = (qtiles - y0) < 65535 ? (qtiles - y0) : 65535;
    b.Qh = a.Qh + y0 * fBQ * 32;
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
      set_error("filter_img2_kernel launch: %s", hipGetErrorString(e));
      return FX_EHIP;
    }
  }
  return check_launch("filter_img2_kernel");
}
#endif  // FX_FILTER_IMG2

// ------------------------------------- tiled image, query tile by LDS-DMA ring
#if FX_FILTER_IMG3
//
// filter_img3_kernel: filter_img2_kernel's tiling (8 waves, wave w owns the
// 32-row tile w of a 256-row tile against all 256 queries, A fragments
// straight from the tiled image into registers) with the query tile moved by
// LDS-DMA (buffer_load ... lds) instead of through registers and ds_write:
//   * the K chunks of the query tile are the same for every row tile, so the
//     chunk sequence runs on across tiles in one ring of FX_I3_QA + 1 slots,
//     FX_I3_QA chunks in flight, one raw s_barrier per chunk behind a counted
//     vmcnt (cdna_hip_programming.md: pipelining across barriers);
//   * 16-B pieces XOR-swizzled by query ((q >> 2) & 3) on the global side:
//     the B-fragment ds_read_b128 are conflict-free without row padding;
//   * the image stream runs on across tiles too: FX_I3_XS register stages,
//     the next tile's first chunks issued as the current tile's last ones
//     are multiplied, so they stream in during its epilogue;
//   * the rows' image sums (and mask words) are loaded at the tile's first
//     chunk, every thread the same count (counted waits stay exact);
//   * appends go to per-query LDS segments (no returning global atomic,
//     which would wait for the prefetched stream: vmcnt retires in order),
//     flushed at the end;
//   * the pass test is packed: per pair of rows one v_pk_fma_f32 gives
//     RN(x - a rv) and one v_pk_add_f32 subtracts b; the sign collects the
//     fail bit (2 instructions per (row, query) instead of 3).
#ifndef FX_I3_QA
#define FX_I3_QA 3   // query chunks in flight (ring of FX_I3_QA + 1 slots)
#endif
#ifndef FX_I3_XS
#define FX_I3_XS 4   // image chunks in flight per wave (register stages; 2 and 3
                     // measured 1-2 % slower, tools/ab_i8x.sh)
#endif
#ifndef FX_I3_SEG
#define FX_I3_SEG 24  // LDS append entries per query (overflow: global slots)
#endif
#ifndef FX_I3_BPF
#define FX_I3_BPF 1   // B-fragment reads of a k-step ahead of its MFMAs (see compute)
#endif
#ifndef FX_I3_XPF
#define FX_I3_XPF 0   // 1: the next tile's first image chunks in flight during the
                      // epilogue (equal with 4 stages, 1-2 % faster with 2)
#endif
#ifndef FX_I3_PAIR
#define FX_I3_PAIR 1  // 1: the ring refilled two chunks at a time, one barrier per
                      // two steps (the ring then holds two pairs; FX_I3_QA unused)
#endif
#ifndef FX_I3_WAVES
#define FX_I3_WAVES 8  // waves per workgroup: 8 (one 256-row workgroup per CU) or 4
                       // (two independent 128-row workgroups per CU)
#endif
constexpr int kI3Waves = FX_I3_WAVES;
constexpr int kI3Threads = 64 * kI3Waves;
constexpr int kI3BM = 32 * kI3Waves;    // rows per workgroup tile (one 32-row tile per wave)
constexpr int kI3Sub = fBM / kI3BM;     // workgroup tiles per fBM-row tile of the phase plan
#ifndef FX_I3_BPC
#define FX_I3_BPC (fWaves / FX_I3_WAVES)  // workgroups per CU in the launch
#endif
constexpr int kI3Slots = FX_I3_QA + 1;
constexpr int kI3QBytes = fBQ * fBK * 2;               // one slot: 16 KB (256 queries)
constexpr int kI3QDmaAll = kI3QBytes / 1024;           // 1-KB DMAs per chunk
// 1-KB DMAs per wave per chunk: every wave the same count, or (64-query tiles:
// 4 KB per chunk) one each on the first kI3QDmaAll waves and none on the rest
constexpr int kI3QDma = kI3QDmaAll >= kI3Waves ? kI3QDmaAll / kI3Waves : 1;
static_assert((kI3QDmaAll >= kI3Waves ? kI3QDma * kI3Waves : kI3QDmaAll) == kI3QDmaAll &&
                  kI3QDmaAll * 1024 == kI3QBytes && fBK == 32,
              "query ring");
static_assert(kI3Sub * kI3BM == fBM && kI3Waves <= fWaves, "workgroup tile");
struct Img3Shared {
  unsigned char qring[kI3Slots][kI3QBytes];
  float rinfo[kI3BM];
  float rterm[kI3BM];
  uint32_t rflags[2][kRowFlagWords];
  f32x4 qtab[fBQ];
  float2 qab[fBQ];
  uint32_t seg[fBQ + 3 * fBQ * FX_I3_SEG];  // counters, then entries {lb key, ub key, row}
  uint32_t segbase[fBQ];
  float rext[kI3BM];  // int8 image: 1 / s of the row
  f32x4 qinf[fBQ];   // int8 image: the query's launch_qprep8 record
  uint32_t rrow[kI3BM];  // int8 image: the global corpus row of the tile row (image8_perm)
};
static_assert(sizeof(Img3Shared) * (fWaves / kI3Waves) <= 160 * 1024,
              "filter_img3_kernel: LDS over 160 KB per CU");

typedef __attribute__((address_space(3))) void* i3_lds_ptr;

template <int N>
__device__ __forceinline__ void i3_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// LDS appends through inline asm: the compiler cannot tell the append
// segments from an LDS-DMA ring, so in a kernel with one it put vmcnt(0)
// before a plain ds_add_rtn / ds_write -- waiting for the ring's chunks in
// flight, about 1-2 us per wave and tile with an append (filter_img8_kernel:
// configs[2]'s F2 ran 1.94 ms with its appends, 1.09 without them).  The
// segments are never DMA targets; the flush reads them behind a barrier.
__device__ __forceinline__ uint32_t lds_add_rtn_u32(uint32_t* p, uint32_t v) {
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)(p);
  uint32_t r;
  asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a), "v"(v) : "memory");
  return r;
}
__device__ __forceinline__ void lds_write1_u32(uint32_t* p, uint32_t x) {
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)(p);
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(x) : "memory");
}
__device__ __forceinline__ void lds_write2_u32(uint2* p, uint32_t x, uint32_t y) {
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint2*)(p);
  asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(uint2{x, y}) : "memory");
}
__device__ __forceinline__ void lds_write3_u32(uint32_t* p, uint32_t x, uint32_t y, uint32_t z) {
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)(p);
  asm volatile("ds_write_b32 %0, %1\n\tds_write_b32 %0, %2 offset:4\n\tds_write_b32 %0, %3 offset:8"
               ::"v"(a), "v"(x), "v"(y), "v"(z) : "memory");
}

// The pass test and appends of one wave's 32-row tile (RT = 1) against all
// kI2QT query tiles; appends into LDS segments (filter_epilogue_seg's layout).
template <int METRIC>
__device__ __forceinline__ void i3_epilogue(const f32x16 (&acc)[kI2QT], const float* rinfo,
                                            const float* rterm, const uint32_t* flags,
                                            const f32x4* qtab, const float2* qab,
                                            const FilterArgs& a, int64_t q0, int64_t r0, int wid,
                                            int h, int l32, uint32_t* seg, int diag) {
  constexpr int SEG = FX_I3_SEG;
  // row j of the lane (accumulator element j) is local row lr0 + (j & 3) + 8 (j >> 2)
  const int lr0 = wid * 32 + 4 * h;
  f32x4 rv4[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) rv4[g] = *reinterpret_cast<const f32x4*>(rinfo + lr0 + 8 * g);
  const uint32_t fmask = flags[wid * 2 + h], smask = flags[16 + wid * 2 + h];
  uint32_t pm[kI2QT];
#pragma unroll
  for (int u = 0; u < kI2QT; ++u) {
    const float2 ab = qab[u * 32 + l32];
    const f32x2 na = {-ab.x, -ab.x}, nb = {-ab.y, -ab.y};
    // fail bit j = sign of RN(RN(x_j - a rv_j) - b): set exactly when x_j -
    // a rv_j rounds below b (NaN passes); bit j enters last-in at bit 0
    uint32_t fail = 0u;
#pragma unroll
    for (int i = 7; i >= 0; --i) {
      const f32x4 r = rv4[i >> 1];
      const f32x2 rp = (i & 1) ? f32x2{r[2], r[3]} : f32x2{r[0], r[1]};
      const f32x2 xp = {acc[u][2 * i], acc[u][2 * i + 1]};
      const f32x2 dd = __builtin_elementwise_fma(na, rp, xp) + nb;
      fail = __builtin_amdgcn_alignbit(fail, __float_as_uint(dd[1]), 31);
      fail = __builtin_amdgcn_alignbit(fail, __float_as_uint(dd[0]), 31);
    }
    pm[u] = (diag & 1) ? 0u : (~fail | fmask) & ~smask & 0xffffu;
    if (q0 + u * 32 + l32 >= a.nq) pm[u] = 0u;
  }
  uint32_t any = 0u;
#pragma unroll
  for (int u = 0; u < kI2QT; ++u) any |= pm[u];
  if (__ballot(any != 0u) == 0ull) return;
  // Appends (a few per wave and tile): per query tile with a pass, a loop
  // over the lane's set bits; the row's accumulator element is selected by
  // a cndmask tree (a dynamic index would put the accumulators in scratch,
  // and a scratch load waits for the whole prefetched stream), its row
  // value re-read from LDS.  static_for over u for the same reason.
  static_for<kI2QT>([&](auto uc) {
    constexpr int u = decltype(uc)::value;
    if (__ballot(pm[u] != 0u) == 0ull) return;
    const int qi = u * 32 + (int)opaque((unsigned)l32);  // (not hoisted: spilled)
    const int64_t gq = q0 + qi;
    uint32_t bits = pm[u];
    uint32_t p = bits != 0u ? lds_add_rtn_u32(&seg[qi], (uint32_t)__popc(bits)) : 0u;
    const f32x4 qc = qtab[qi];
    const float qc1 = qc[0], qc0 = qc[1], qA = qc[2], qB = qc[3];
    const bool fq = !(qA <= 3.4e38f);
    uint32_t gp = ~0u;
    while (bits != 0u) {
      const int j = __builtin_ctz(bits);
      const uint32_t rest = bits;
      bits &= bits - 1u;
      // (bit-field selects, v_bfi_b32: a ?: select tree is turned back into
      // a dynamic index, i.e. scratch)
      auto pick = [](float lo, float hi, uint32_t m) {
        return __uint_as_float((__float_as_uint(hi) & m) | (__float_as_uint(lo) & ~m));
      };
      const uint32_t m0 = 0u - ((uint32_t)j & 1u), m1 = 0u - (((uint32_t)j >> 1) & 1u);
      const uint32_t m2 = 0u - (((uint32_t)j >> 2) & 1u), m3 = 0u - (((uint32_t)j >> 3) & 1u);
      float v8[8], v4[4], v2[2];
#pragma unroll
      for (int i = 0; i < 8; ++i) v8[i] = pick(acc[u][2 * i], acc[u][2 * i + 1], m0);
#pragma unroll
      for (int i = 0; i < 4; ++i) v4[i] = pick(v8[2 * i], v8[2 * i + 1], m1);
#pragma unroll
      for (int i = 0; i < 2; ++i) v2[i] = pick(v4[2 * i], v4[2 * i + 1], m2);
      const float x = pick(v2[0], v2[1], m3);
      const int lr = lr0 + (j & 3) + 8 * (j >> 2);
      const float rv = rinfo[lr];
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
        const float rt = rterm[lr];
        const float dist = fmaf(x * rt, qc1, 0.5f);
        const float e = fmaf(qB, rt, qA);
        lb = dist - e;
        ub = dist + e;
      }
      if (fq || rv != rv) {  // forced: below / above every key
        lb = -__builtin_inff();
        ub = __builtin_nanf("");
      }
      const uint32_t grow = (uint32_t)(a.row_base + r0) + (uint32_t)lr;
      if (p < (uint32_t)SEG) {
        lds_write3_u32(seg + fBQ + 3 * (qi * SEG + p), order_key(lb), order_key(ub), grow);
      } else {  // rare: past the segment, global slots for the lane's remaining passes
        if (gp == ~0u) gp = atomicAdd(&a.count[gq * kCountStride], (uint32_t)__popc(rest));
        if (gp < (uint32_t)a.cap) {
          const size_t slot = (size_t)gq * a.cap + gp;
          if (a.cand_ub != nullptr) {
            a.cand[slot] = make_comp(lb, grow);
            a.cand_ub[slot] = make_comp(ub, grow);
          } else {
            a.cand[slot] = make_comp(ub, grow);
          }
        }
        ++gp;
      }
      ++p;
    }
  });
}

// ------------------------------------------------------ int8 filter image
//
// The int8 image (launch_image8) halves the image stream again and runs on
// v_mfma_i32_32x32x32_i8 (twice the fp16 rate): per row a scale s, x~ =
// rint(x / s) in [-127, 127], w = |x~|, e >= |x - s x~|, v = e / s; per query
// the same with s_q, w_q, e_q (launch_qprep8).  Both are scaled so that w,
// w_q <= 2048, so the exact integer product I = x~ . q~ has |I| <= 2^22.
// With D = x . q, exactly:  D - s s_q I = (x - s x~) . q + s x~ . (q - s_q q~),
//   |D - s s_q I| <= s s_q (v P + w R),  P = |q| / s_q,  R = e_q / s_q
// (IP also carries the scan's f32 summation error g |x||q|, g = (d + 2) 2^-24
// with 1 % slack, into P and R; cosine and L2 carry it in their constants).
// With kappa = kI8Kappa and R' = max(R, P / kappa) (kept by the query),
// v P + w R <= (w + kappa v) R' = omega R': omega is the row's one error
// value (launch_image8).  Per metric, with M = 12582912 + I (the accumulator
// starts at the bits of 1.5 * 2^23, so the i32 sum read as a float is exactly
// M for |I| <= 2^22: no conversion), a pair can reach the threshold T only if
//   IP   I + omega R' + (1/s) (T / s_q)                    >= 0
//   cos  I + omega R' - (N / s) (1 - 2T - 2c) N_q / s_q    >= 0   (N = max(|x|, 1e-12))
//   L2   I + omega R' - (n^2 / s) / (2 s_q) - (1/s) (n_q^2 - T^2 (1 + 2^-20) / (1 - g2)) / (2 s_q) >= 0
// c = 3 g + 16 u and g2 = 2 g + 8 u cover the scan's own roundings (u = 2^-24;
// knn_batch.hip exact_distance16: dot and norms in f32, one division).  Each
// per-query coefficient carries a relative slack >= 16 u (the roundings of the
// products and sums of the test) and the test compares with 12582912 - 8.
// The appends' [lb, ub] (i8_bounds) are evaluated in f32 from the same terms,
// each widened outward by 16 u of the magnitudes it was computed from (every
// rounding on the way is relative to a term it is added to, at most ~8 u).
// A non-finite row or query, or one whose scaled norm would exceed 2048, is
// forced through (omega or R' not finite).
constexpr float kI8Magic = 12582912.f;   // 1.5 * 2^23: bits 0x4B400000
constexpr float kI8C0 = 12582912.f - 8.f;

// Per query {R', c1, c2, 0} of the int8 pass test
//   M + omega R' + y1 c1 + y2 c2 >= kI8C0
// with the row values y1 (IP 1/s, cosine N/s, L2 n^2/s) and y2 (L2 1/s).
// No threshold yet (T NaN) or a forced query: R' = +inf (everything passes).
template <int METRIC>
__device__ __forceinline__ void i8_query_table(const FilterArgs& a, int64_t q0, f32x4* qtab,
                                               f32x4* qinf, int tid, int nthreads) {
  const float u = 5.9604644775390625e-08f;
  const float g = (float)(a.d + 2) * u * 1.01f;
  for (int i = tid; i < fBQ; i += nthreads) {
    const int64_t gq = q0 + i;
    f32x4 c = f32x4(0.f), qi = f32x4(0.f);
    if (gq < a.nq) {
      qi = *reinterpret_cast<const f32x4*>(a.qinfo + gq * kI8QInfo);  // {s_q, R', n_q^2, |q|}
      float tf = key_float((uint32_t)(a.thr[gq] >> 32));
      // the upper-bound test (ub_test): -R' below, T widened by 2^-14
      // relative (the rows that set T pass again)
      if (a.ub_test) tf += fabsf(tf) * 6.103515625e-05f;
      const float sq = qi[0];
      c[0] = qi[1];
      if constexpr (METRIC == 1) {
        const float t = tf / sq;
        c[1] = t + 16.f * u * fabsf(t);
      } else if constexpr (METRIC == 2) {
        const float cc = 3.f * g + 16.f * u;
        const float K = (1.f - 2.f * tf - 2.f * cc) * (fmaxf(qi[3], 1e-12f) / sq);
        c[1] = -K + (g + 16.f * u) * fabsf(K);
      } else {
        const float g2 = 2.f * g + 8.f * u;
        const float L1 = 0.5f / sq;
        const float t2 = tf * tf * (1.f + 9.5367431640625e-07f) / (1.f - g2);
        const float L0 = (qi[2] * (1.f - 4.f * u) - t2) * L1;
        c[1] = -L1 * (1.f - g - 16.f * u);
        c[2] = -L0 + 16.f * u * fabsf(L0);
      }
      if (tf != tf || !(c[0] <= 3.4e38f))
        c = f32x4{__builtin_inff(), 0.f, 0.f, 0.f};
      else if (a.ub_test)
        c[0] = -c[0];
    }
    qtab[i] = c;
    qinf[i] = qi;
  }
}

// [lb, ub] of an appended (row, query) pair of the int8 filter from M, the
// row's {omega, y1, 1/s} (i8_note_row) and the query's launch_qprep8 record,
// in f32 with outward slack: every rounding below is relative to a term it
// is added to (at most ~8 u each), so each bound is widened by 16 u of the
// magnitudes it was computed from.
template <int METRIC>
__device__ __forceinline__ void i8_bounds(float m, float om, float y1, float is, f32x4 qi, int d,
                                          float& lb, float& ub) {
  if (om != om) {  // forced row: below / above every key
    lb = -__builtin_inff();
    ub = __builtin_nanf("");
    return;
  }
  const float u = 5.9604644775390625e-08f;
  const float g = (float)(d + 2) * u * 1.01f;
  const float I = m - kI8Magic;  // exact
  const float E = fmaf(om * qi[1], 8.f * u, om * qi[1]) + 4.f;
  const float s = 1.f / is;
  const float sig = s * qi[0];
  const float a1 = I + E, a2 = I - E;
  if constexpr (METRIC == 1) {
    const float lo = -sig * a1, hi = -sig * a2;
    lb = lo - 16.f * u * fabsf(lo);
    ub = hi + 16.f * u * fabsf(hi);
  } else if constexpr (METRIC == 2) {
    const float c = 3.f * g + 32.f * u;
    const float den = fmaxf(y1 * s, 1e-12f) * fmaxf(qi[3], 1e-12f);
    const float r1 = sig * a1 / den, r2 = sig * a2 / den;
    lb = 0.5f - 0.5f * r1 - c - 16.f * u * (1.f + fabsf(r1));
    ub = 0.5f - 0.5f * r2 + c + 16.f * u * (1.f + fabsf(r2));
  } else {
    const float g2 = 2.f * g + 8.f * u;
    const float n2 = y1 * s;
    const float alo = n2 * (1.f - g - 16.f * u) + qi[2] * (1.f - 4.f * u);
    const float ahi = n2 * (1.f + g + 16.f * u) + qi[2] * (1.f + 4.f * u);
    const float t1 = 2.f * sig * a1, t2 = 2.f * sig * a2;
    const float lo2 = (1.f - g2) * (alo - t1) - 16.f * u * (alo + fabsf(t1));
    const float hi2 = (1.f + g2) * (ahi - t2) + 16.f * u * (ahi + fabsf(t2));
    lb = sqrtf(fmaxf(lo2, 0.f)) * (1.f - 4.f * u);
    ub = sqrtf(fmaxf(hi2, 0.f)) * (1.f + 4.f * u);
  }
  if (lb != lb) lb = -__builtin_inff();  // (a non-finite query: R' = inf)
  if (ub != ub) ub = __builtin_nanf("");
}

// One row's values for the int8 epilogue: omega (NaN: forced), y1 and 1/s,
// and its flags (filter_note_row's words)
__device__ __forceinline__ void i8_note_row(float* rinfo, float* rterm, float* rext,
                                            uint32_t* flags, int lr, float om, float y1, float is,
                                            bool ok) {
  rinfo[lr] = om;
  rterm[lr] = y1;
  rext[lr] = is;
  int word, bit;
  filter_row_bit<1>(lr, word, bit);
  if (!ok) atomicOr(&flags[16 + word], 1u << bit);
  else if (om != om) atomicOr(&flags[word], 1u << bit);
}

// i3_epilogue for the int8 image: the packed pass test above (2 or 3
// v_pk_fma_f32 and one v_pk_add_f32 per two pairs), appends with i8_bounds
// all-pass phases of at most this many tiles reserve fixed slots even when
// the slice shares its segments (i8_epilogue)
constexpr int64_t kAllPassSlotTiles = 64;
template <int METRIC>
__device__ __forceinline__ void i8_epilogue(const f32x16 (&acc)[kI2QT], const float* rinfo,
                                            const float* rterm, const float* rext,
                                            const uint32_t* rrow, const uint32_t* flags,
                                            const f32x4* qtab, const f32x4* qinf,
                                            const FilterArgs& a, int64_t q0, int wid, int h,
                                            int l32, uint32_t* seg, int diag,
                                            int segcap = FX_I3_SEG) {
  const int lr0 = wid * 32 + 4 * h;
  const uint32_t fmask = flags[wid * 2 + h], smask = flags[16 + wid * 2 + h];
  // row groups g of 4 rows outside (their values read once from LDS), query
  // tiles inside; fail bit j = 4 g + i enters last-in at bit 0, so g and i
  // run down
  uint32_t fail[kI2QT];
#pragma unroll
  for (int u = 0; u < kI2QT; ++u) fail[u] = 0u;
  const f32x2 nc0 = {-kI8C0, -kI8C0};
#pragma unroll
  for (int g = 3; g >= 0; --g) {
    const f32x4 om = *reinterpret_cast<const f32x4*>(rinfo + lr0 + 8 * g);
    const f32x4 y1 = *reinterpret_cast<const f32x4*>(rterm + lr0 + 8 * g);
    f32x4 y2 = f32x4(0.f);
    if constexpr (METRIC == 0) y2 = *reinterpret_cast<const f32x4*>(rext + lr0 + 8 * g);
#pragma unroll
    for (int u = 0; u < kI2QT; ++u) {
      const f32x4 co = qtab[u * 32 + l32];
      const f32x2 ra = {co[0], co[0]}, c1 = {co[1], co[1]}, c2 = {co[2], co[2]};
#pragma unroll
      for (int hp = 1; hp >= 0; --hp) {  // rows 4 g + 2 hp, + 1
        const int i = 2 * g + hp;
        const f32x2 xp = {acc[u][2 * i], acc[u][2 * i + 1]};
        const f32x2 op = hp ? f32x2{om[2], om[3]} : f32x2{om[0], om[1]};
        const f32x2 p1 = hp ? f32x2{y1[2], y1[3]} : f32x2{y1[0], y1[1]};
        f32x2 t = __builtin_elementwise_fma(op, ra, xp);
        t = __builtin_elementwise_fma(p1, c1, t);
        if constexpr (METRIC == 0) {
          const f32x2 p2 = hp ? f32x2{y2[2], y2[3]} : f32x2{y2[0], y2[1]};
          t = __builtin_elementwise_fma(p2, c2, t);
        }
        const f32x2 dd = t + nc0;
        fail[u] = __builtin_amdgcn_alignbit(fail[u], __float_as_uint(dd[1]), 31);
        fail[u] = __builtin_amdgcn_alignbit(fail[u], __float_as_uint(dd[0]), 31);
      }
    }
  }
  uint32_t pm[kI2QT];
  // (all_pass: every live row, whatever the test says: with R' = inf a zero
  // row's 0 * inf is a NaN whose sign decides the bit)
  const uint32_t force = a.all_pass ? ~0u : fmask;
#pragma unroll
  for (int u = 0; u < kI2QT; ++u) {
    pm[u] = (diag & 1) ? 0u : (~fail[u] | force) & ~smask & 0xffffu;
    if (q0 + u * 32 + l32 >= a.nq) pm[u] = 0u;
  }
  if (a.all_pass && (segcap <= FX_I3_SEG || a.num_tiles <= kAllPassSlotTiles)) {
                     // no threshold yet (first phase): every live pair, slots reserved
                     // per lane and query, accumulators indexed statically (a slice
                     // of few live queries over a large first sample, k ~ 1 000,
                     // appends through its segments below instead: its whole sample
                     // otherwise meets in one global counter, ~3 K atomics; a small
                     // one, k = 100's 20 tiles, is faster through the slots)
    static_for<kI2QT>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      const uint32_t bits = pm[u];
      if (__ballot(bits != 0u) == 0ull) return;
      const int qi = u * 32 + (int)opaque((unsigned)l32);
      const int64_t gq = q0 + qi;
      uint32_t p = bits != 0u ? atomicAdd(&a.count[gq * kCountStride], (uint32_t)__popc(bits)) : 0u;
      const f32x4 qrec = qinf[qi];
      static_for<16>([&](auto jc) {
        constexpr int jj = decltype(jc)::value;
        if (!((bits >> jj) & 1u)) return;
        // (opaque: 16 rows' LDS offsets hoisted to the kernel start were spilled)
        const int lr = (int)opaque((unsigned)lr0) + (jj & 3) + 8 * (jj >> 2);
        float lb, ub;
        i8_bounds<METRIC>(acc[u][jj], rinfo[lr], rterm[lr], rext[lr], qrec, a.d, lb, ub);
        if (p < (uint32_t)a.cap) {
          const uint32_t grow = rrow[lr];
          const size_t slot = (size_t)gq * a.cap + p;
          if (a.cand_ub != nullptr) {
            a.cand[slot] = make_comp(lb, grow);
            a.cand_ub[slot] = make_comp(ub, grow);
          } else {
            a.cand[slot] = make_comp(ub, grow);
          }
        }
        ++p;
      });
    });
    return;
  }
  uint32_t any = 0u;
#pragma unroll
  for (int u = 0; u < kI2QT; ++u) any |= pm[u];
  if (__ballot(any != 0u) == 0ull) return;
  static_for<kI2QT>([&](auto uc) {
    constexpr int u = decltype(uc)::value;
    if (__ballot(pm[u] != 0u) == 0ull) return;
    const int qi = u * 32 + (int)opaque((unsigned)l32);  // (not hoisted: spilled)
    const int64_t gq = q0 + qi;
    uint32_t bits = pm[u];
    uint32_t p = bits != 0u ? lds_add_rtn_u32(&seg[qi], (uint32_t)__popc(bits)) : 0u;
    const f32x4 qrec = qinf[qi];
    uint32_t gp = ~0u;
    while (bits != 0u) {
      const int j = __builtin_ctz(bits);
      const uint32_t rest = bits;
      bits &= bits - 1u;
      auto pick = [](float lo, float hi, uint32_t m) {
        return __uint_as_float((__float_as_uint(hi) & m) | (__float_as_uint(lo) & ~m));
      };
      const uint32_t m0 = 0u - ((uint32_t)j & 1u), m1 = 0u - (((uint32_t)j >> 1) & 1u);
      const uint32_t m2 = 0u - (((uint32_t)j >> 2) & 1u), m3 = 0u - (((uint32_t)j >> 3) & 1u);
      float v8[8], v4[4], v2[2];
#pragma unroll
      for (int i = 0; i < 8; ++i) v8[i] = pick(acc[u][2 * i], acc[u][2 * i + 1], m0);
#pragma unroll
      for (int i = 0; i < 4; ++i) v4[i] = pick(v8[2 * i], v8[2 * i + 1], m1);
#pragma unroll
      for (int i = 0; i < 2; ++i) v2[i] = pick(v4[2 * i], v4[2 * i + 1], m2);
      const float x = pick(v2[0], v2[1], m3);
      const int lr = lr0 + (j & 3) + 8 * (j >> 2);
      float lb, ub;
      i8_bounds<METRIC>(x, rinfo[lr], rterm[lr], rext[lr], qrec, a.d, lb, ub);
      const uint32_t grow = rrow[lr];
      if (p < (uint32_t)segcap) {
        lds_write3_u32(seg + fBQ + 3 * (qi * segcap + p), order_key(lb), order_key(ub), grow);
      } else {  // rare: past the segment, global slots for the lane's remaining passes
        if (gp == ~0u) gp = atomicAdd(&a.count[gq * kCountStride], (uint32_t)__popc(rest));
        if (gp < (uint32_t)a.cap) {
          const size_t slot = (size_t)gq * a.cap + gp;
          if (a.cand_ub != nullptr) {
            a.cand[slot] = make_comp(lb, grow);
            a.cand_ub[slot] = make_comp(ub, grow);
          } else {
            a.cand[slot] = make_comp(ub, grow);
          }
        }
        ++gp;
      }
      ++p;
    }
  });
}

template <int METRIC, bool I8>
__global__ void __launch_bounds__(kI3Threads, 2) filter_img3_kernel(FilterArgs a) {
  constexpr int XS = FX_I3_XS, SEG = FX_I3_SEG;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  Img3Shared* sh = reinterpret_cast<Img3Shared*>(smem);
#ifdef FX_DIAG_BUILD  // FX_FILTER_DIAG: 1 no appends, 2 no epilogue, 4 no MFMA,
                      // 8 no query DMA, 16 no step barrier, 32 no image loads
  const int diag = a.diag;
#else
  constexpr int diag = 0;
#endif
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, l32 = lane & 31;
  const int64_t q0 = (int64_t)blockIdx.y * fBQ;
  // chunks per tile, padded to a multiple of the register stages (past the
  // row end the image reads zeros and the query tile is zero-padded to dq)
  // (int8 image: 64 components per chunk, 32 per k-step, the same bytes)
  constexpr int CK = I8 ? 2 * fBK : fBK;
  const int nch = ((a.d + CK - 1) / CK + XS - 1) / XS * XS;
  const int ksteps = I8 ? (a.d + 31) / 32 : (a.d + 15) / 16;
  const int64_t ntile32 = (a.n + 31) / 32;
  // workgroup tiles: kI3Sub per fBM-row tile of the plan (a.tile_start, ...)
  const int64_t ntiles = a.num_tiles * kI3Sub;
  auto tile_r0 = [&](int64_t ti) {
    return (a.tile_start + (ti / kI3Sub) * a.tile_stride) * fBM + (ti % kI3Sub) * kI3BM;
  };
  if ((int64_t)blockIdx.x >= ntiles) return;
  if (a.skip_full) {  // every query of the tile predicted to overflow: nothing to do
    bool full = true;
    for (int q = tid; q < fBQ; q += kI3Threads)
      if (q0 + q < a.nq && a.count[(q0 + q) * kCountStride] <= (uint32_t)a.cap) full = false;
    if (__syncthreads_and(full)) return;
  }
  if constexpr (I8)
    i8_query_table<METRIC>(a, q0, sh->qtab, sh->qinf, tid, kI3Threads);
  else
    filter_query_table<METRIC>(a, q0, sh->qtab, sh->qab, tid, kI3Threads);
  for (int q = tid; q < fBQ; q += kI3Threads) sh->seg[q] = 0u;  // (ordered by the first barrier)
  // the ring starts zeroed (a slot whose DMA is dropped then holds finite values)
  for (int i = tid; i < kI3Slots * kI3QBytes / 16; i += kI3Threads)
    reinterpret_cast<i32x4*>(sh->qring)[i] = i32x4(0);
  __syncthreads();

  // the query tile, blocked by 32 components (FilterArgs::Qh); chunk c of
  // query q is 64 B at (c * qstride + q) * 64
  const __amdgpu_buffer_rsrc_t qr = [&] {
    const uint64_t qp = reinterpret_cast<uint64_t>(a.Qh + q0 * 32);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)qp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(qp >> 32));
    const int nb = __builtin_amdgcn_readfirstlane(
        (int)(((int64_t)(a.dq / 32 - 1) * a.qstride + fBQ) * 64));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                             nb, 0x00020000);
  }();
  // this lane's piece of each of the wave's DMAs: query 16 j + lane / 4, slot
  // piece lane % 4 holding global piece (lane % 4) ^ ((q >> 2) & 3)
  uint32_t qv[kI3QDma];
#pragma unroll
  for (int i = 0; i < kI3QDma; ++i) {
    const int j = wid * kI3QDma + i;
    const int q = 16 * j + (lane >> 2);
    qv[i] = (uint32_t)(q * 64 + (((lane & 3) ^ ((q >> 2) & 3)) * 16));
  }
  // (chunks past the query tile's padding, when nch is padded to the
  // stages: an offset beyond the buffer, the DMA is dropped and the slot
  // keeps finite values of an earlier chunk, multiplied by zero image rows)
  const int qchunks = a.dq / CK;
  auto issue_q = [&](int c, int slot) {
    if (diag & 8) return;
    if (kI3QDmaAll < kI3Waves && wid >= kI3QDmaAll) return;  // (wave-uniform)
    unsigned char* st = sh->qring[slot];
#pragma unroll
    for (int i = 0; i < kI3QDma; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(qr, (i3_lds_ptr)(st + (wid * kI3QDma + i) * 1024), 16,
                                               c < qchunks ? qv[i] : 0x7fff0000u,
                                               (int)(c * a.qstride * 64), 0, 0);
  };
  // this wave's 32-row tile of the row tile at step iteration ti: its
  // k-steps, one KB each (a tile past the end: an empty descriptor, zeros)
  auto x_rsrc = [&](int64_t ti) {
    const int64_t t32 = tile_r0(ti) / 32 + wid;
    const int64_t live = (ti < ntiles && t32 < ntile32) ? 1 : 0;
    const unsigned char* base = reinterpret_cast<const unsigned char*>(a.X) +
                                (live ? t32 : 0) * (int64_t)ksteps * 1024;
    const uint64_t xp = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)xp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(xp >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)(live * ksteps * 1024));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                             nb, 0x00020000);
  };
  const uint32_t xl = (uint32_t)opaque(lane) * 16u;
  typedef f16x8 XA[kI2KS];
  auto load_x = [&](XA& xa, __amdgpu_buffer_rsrc_t xr, int c) {
    if (diag & 32) {
#pragma unroll
      for (int s = 0; s < kI2KS; ++s) xa[s] = f16x8((_Float16)0.f);
      return;
    }
#pragma unroll
    for (int s = 0; s < kI2KS; ++s) {
      const int ks = c * kI2KS + s;  // wave-uniform: past the row end reads zeros
      const uint32_t off = ks < ksteps ? xl : 0x7fff0000u;
      xa[s] = __builtin_bit_cast(
          f16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, off, ks * 1024, 2 /* nt */));
    }
  };
  // B fragment of query tile u, k-step s of a slot: query Q = 32 u + l32,
  // global piece 2 s + h at its swizzled place
  uint32_t bq[kI2KS];
#pragma unroll
  for (int s = 0; s < kI2KS; ++s) {
    const int Q = (int)opaque((unsigned)l32);
    bq[s] = (uint32_t)(Q * 64 + (((2 * s + h) ^ ((Q >> 2) & 3)) * 16));
  }
  f32x16 acc[kI2QT];
  // a tile's first k-step takes its accumulator input from this constant
  // (int8: the bits of 1.5 * 2^23, see "int8 filter image"; fp16: zeros)
  // instead of 128 moves per tile into the accumulators
  const f32x16 acc0 = f32x16(I8 ? kI8Magic : 0.f);
  // FIRST: the tile's first chunk (its k-step 0 starts from acc0)
  auto compute = [&](const XA& xa, int slot, auto first) {
    constexpr bool FIRST = decltype(first)::value;
    if (diag & 4) {  // (diagnostics: no MFMA; the row loads stay live)
      if (xa[0][0] == (_Float16)1.2345f && xa[kI2KS - 1][7] == (_Float16)2.f) a.count[0] = 7;
      if (FIRST) {
#pragma unroll
        for (int u = 0; u < kI2QT; ++u) acc[u] = acc0;
      }
      return;
    }
    const unsigned char* st = sh->qring[slot];
    // B fragments of a k-step read into their own registers before its
    // MFMAs (FX_I3_BPF 1; 2: both k-steps' first): left to itself, hipcc
    // read each fragment into one register set right before its MFMA and
    // waited lgkmcnt(0) in between, so every MFMA paid a full LDS latency
    auto mfma = [&](int u, const f16x8& xv, const f16x8& bv, bool start) {
      const f32x16 cin = start ? acc0 : acc[u];
      if constexpr (I8) {
        typedef int i32x16 __attribute__((ext_vector_type(16)));
        acc[u] = __builtin_bit_cast(f32x16, __builtin_amdgcn_mfma_i32_32x32x32_i8(
            __builtin_bit_cast(i32x4, xv), __builtin_bit_cast(i32x4, bv),
            __builtin_bit_cast(i32x16, cin), 0, 0, 0));
      } else {
        acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xv, bv, cin, 0, 0, 0);
      }
    };
#if FX_I3_BPF != 0
    // (query tile u sits 32 x 64 B further: (Q + 32 u) has the same swizzle)
    auto read_b = [&](f16x8 (&bv)[kI2QT], int s) {
#pragma unroll
      for (int u = 0; u < kI2QT; ++u)
        bv[u] = *reinterpret_cast<const f16x8*>(st + bq[s] + u * 32 * 64);
    };
#endif
#if FX_I3_BPF == 0
    static_for<kI2KS>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
#pragma unroll
      for (int u = 0; u < kI2QT; ++u) {
        const f16x8 bv = *reinterpret_cast<const f16x8*>(st + bq[s] + u * 32 * 64);
        mfma(u, xa[s], bv, FIRST && s == 0);
      }
    });
#elif FX_I3_BPF == 1
    static_for<kI2KS>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      f16x8 bv[kI2QT];
      read_b(bv, s);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < kI2QT; ++u) mfma(u, xa[s], bv[u], FIRST && s == 0);
      __builtin_amdgcn_sched_barrier(0);
    });
#else
    static_assert(kI2KS == 2, "FX_I3_BPF 2: two k-steps per chunk");
    f16x8 b0[kI2QT], b1[kI2QT];
    read_b(b0, 0);
    read_b(b1, 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kI2QT; ++u) mfma(u, xa[0], b0[u], FIRST);
#pragma unroll
    for (int u = 0; u < kI2QT; ++u) mfma(u, xa[1], b1[u], false);
    __builtin_amdgcn_sched_barrier(0);
#endif
  };

  // ---- prologue: query chunks 0 .. QA-1 and image chunks 0 .. XS-1 of the
  // first tile in flight
  int qc = 0, qslot = 0;  // next query chunk to issue and its slot
  static_assert(!FX_I3_PAIR || (kI3Slots == 4 && XS % 2 == 0), "FX_I3_PAIR: two pairs, even stages");
#pragma unroll
  for (int i = 0; i < (FX_I3_PAIR ? 2 : FX_I3_QA); ++i) {
    issue_q(qc, qslot);
    qc = qc + 1 == nch ? 0 : qc + 1;
    qslot = qslot + 1 == kI3Slots ? 0 : qslot + 1;
  }
  XA xa[XS];
  int64_t xt = blockIdx.x;  // tile (iteration index) of the next image chunk to load
  int xc = 0;
  __amdgpu_buffer_rsrc_t xr = x_rsrc(xt);
  static_for<XS>([&](auto sc) {
    load_x(xa[decltype(sc)::value], xr, xc);
    if (++xc == nch) {
      xc = 0;
      xt += gridDim.x;
      xr = x_rsrc(xt);
    }
  });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (once: the prologue's order differs)
  int rslot = 0;  // slot of the query chunk the next step reads
  int par = 0;
  const int lr = tid & (kI3BM - 1);  // the row this thread notes (threads >= kI3BM: duplicates)
  for (int64_t ti = blockIdx.x; ti < ntiles; ti += gridDim.x, par ^= 1) {
    const int64_t r0 = tile_r0(ti);
    if (tid < kRowFlagWords) sh->rflags[par][tid] = 0u;  // (read two tiles back)
    std::conditional_t<I8, f32x4, float> rsum = {};
    uint32_t mword = 0u;
    // one K step: multiply chunk c + S, then (LOAD) refill its register
    // stage with the chunk XS steps ahead (the next tile's first chunks at
    // the end of a tile, FX_I3_XPF)
    auto step = [&](int c, auto sc, auto ld, auto first) {
      constexpr int S = decltype(sc)::value;
      // query chunk c + S landed (this wave's DMAs; vmcnt retires in issue
      // order, and the loads issued after it are QA - 1 steps' DMAs plus the
      // image chunks of the QA steps from its own: none in a group that loads
      // nothing, i.e. the tile's last group without FX_I3_XPF, where only the
      // steps before the group's start loaded; extra loads, e.g. the rows'
      // terms, only make the wait stronger), and every wave done with the
      // slot refilled next
      constexpr bool LD = decltype(ld)::value;
      if constexpr (FX_I3_PAIR) {
        // even steps only (nch is a multiple of XS, so the step parity is
        // S's): the pair (c + S, c + S + 1) was issued two steps back, and
        // after it only image chunks: the two steps' own (none in a tile's
        // last group), or at a tile's first group the post-epilogue stages
        if constexpr (S % 2 == 0) {
          constexpr int kN = S == 0 ? (decltype(first)::value && !FX_I3_XPF ? XS * kI2KS : 2 * kI2KS)
                                    : (LD ? 2 * kI2KS : 0);
          if (diag & 16)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          else
            i3_wait_barrier<kN>();
#pragma unroll
          for (int i = 0; i < 2; ++i) {  // into the pair every wave finished before the barrier
            issue_q(qc, qslot);
            qc = qc + 1 == nch ? 0 : qc + 1;
            qslot = qslot + 1 == kI3Slots ? 0 : qslot + 1;
          }
        }
      } else {
      constexpr int kXAfter = LD ? FX_I3_QA : (FX_I3_QA > S ? FX_I3_QA - S : 0);
      if (diag & 16)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else
        i3_wait_barrier<(FX_I3_QA - 1) * kI3QDma + kXAfter * kI2KS>();
      issue_q(qc, qslot);
      qc = qc + 1 == nch ? 0 : qc + 1;
      qslot = qslot + 1 == kI3Slots ? 0 : qslot + 1;
      }
      if constexpr (decltype(first)::value && S == 0) {  // the rows' image sums and mask words of this tile
        const int64_t row = r0 + lr < a.n ? r0 + lr : a.n - 1;
        if constexpr (I8)
          rsum = *reinterpret_cast<const f32x4*>(a.rowinfo + row * kI8RowInfo);
        else
          rsum = a.rowinfo[row];
        // (int8 image: the mask bit of the corpus row the image row holds)
        int64_t mrow = row;
        if constexpr (I8) mrow = perm_row(a.perm_a, a.n, row);
        // (both kernel arguments: global loads; a pointer to a __device__
        // constant made a flat load, which counts in lgkmcnt too, and the
        // step's LDS waits then waited for it)
        const bool masked = a.mask != nullptr;
        const uint32_t* mp = masked ? a.mask + (mrow >> 5)
                                    : reinterpret_cast<const uint32_t*>(a.rowinfo) + row * (I8 ? kI8RowInfo : 1);
        mword = *mp | (masked ? 0u : ~0u);
        if constexpr (I8) mword = masked ? (mword >> (mrow & 31)) << (row & 31) : mword;
      }
      compute(xa[S], rslot, std::bool_constant<decltype(first)::value && S == 0>{});
      rslot = rslot + 1 == kI3Slots ? 0 : rslot + 1;
      if constexpr (decltype(ld)::value) {
        load_x(xa[S], xr, xc);
        if (++xc == nch) {
          xc = 0;
          xt += gridDim.x;
          xr = x_rsrc(xt);
        }
      }
    };
    using Load = std::true_type;
    using Xpf = std::integral_constant<bool, FX_I3_XPF>;
    using First = std::true_type;
    using Later = std::false_type;
    // the first chunk group peeled (its first k-step starts from acc0)
    if (nch > XS) {
      static_for<XS>([&](auto sc) { step(0, sc, Load{}, First{}); });
      int c = XS;
      for (; c + XS < nch; c += XS)
        static_for<XS>([&](auto sc) { step(c, sc, Load{}, Later{}); });
      static_for<XS>([&](auto sc) { step(c, sc, Xpf{}, Later{}); });
    } else {
      static_for<XS>([&](auto sc) { step(0, sc, Xpf{}, First{}); });
    }
    if (tid < kI3BM) {  // one thread per row: bound factor, flags
      // (the row index recomputed here from opaque(tid): hoisted out of the
      // tile loop, its flag bit was spilled and reloaded behind a vmcnt(0))
      const int lr = (int)opaque((unsigned)tid);
      const int64_t row = r0 + lr;
      bool ok = row < a.n && ((mword >> (row & 31)) & 1u);
      if constexpr (I8) {  // {omega, 1/s, N/s, n^2/s}
        const float y1 = METRIC == 1 ? rsum[1] : METRIC == 2 ? rsum[2] : rsum[3];
        i8_note_row(sh->rinfo, sh->rterm, sh->rext, sh->rflags[par], lr, rsum[0], y1, rsum[1], ok);
        sh->rrow[lr] = (uint32_t)a.row_base + (row < a.n ? perm_row(a.perm_a, a.n, row) : 0u);
      } else {
      const float s = ok ? rsum : 0.f;
      float rv;
      if constexpr (METRIC == 0) {
        rv = s;
      } else if constexpr (METRIC == 1) {
        rv = sqrtf(s);
      } else {
        rv = fmaxf(sqrtf(s), 1e-12f);
      }
      if (!(s <= 3.4e38f)) rv = __builtin_nanf("");
      filter_note_row<METRIC, 1>(sh->rinfo, sh->rterm, sh->rflags[par], lr, rv, ok);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (diag & 2) {
      if (acc[0][0] == 1.2345f) a.count[0] = 7;
    } else {
      if constexpr (I8)
        i8_epilogue<METRIC>(acc, sh->rinfo, sh->rterm, sh->rext, sh->rrow, sh->rflags[par],
                            sh->qtab, sh->qinf, a, q0, wid, h, l32, sh->seg, diag);
      else
        i3_epilogue<METRIC>(acc, sh->rinfo, sh->rterm, sh->rflags[par], sh->qtab, sh->qab, a, q0,
                            r0, wid, h, l32, sh->seg, diag);
    }
    if constexpr (!FX_I3_XPF) {  // the next tile's first chunks, after the epilogue
      static_for<XS>([&](auto sc) {
        load_x(xa[decltype(sc)::value], xr, xc);
        if (++xc == nch) {
          xc = 0;
          xt += gridDim.x;
          xr = x_rsrc(xt);
        }
      });
    }
  }
  // the ring's and the stream's last loads (past the end) land before the
  // workgroup's LDS is released; then the segments go out
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  filter_flush_segments<SEG, kI3Threads>(sh->seg, sh->segbase, a, q0, tid);
}

static int launch_img3(const FilterArgs& a, int metric, hipStream_t stream) {
  const size_t smem = sizeof(Img3Shared);
  const void* fn =
      a.img8 ? (metric == FX_METRIC_COS  ? (const void*)filter_img3_kernel<2, true>
                : metric == FX_METRIC_IP ? (const void*)filter_img3_kernel<1, true>
                                         : (const void*)filter_img3_kernel<0, true>)
             : (metric == FX_METRIC_COS  ? (const void*)filter_img3_kernel<2, false>
                : metric == FX_METRIC_IP ? (const void*)filter_img3_kernel<1, false>
                                         : (const void*)filter_img3_kernel<0, false>);
  if (int rc = allow_lds(fn)) return rc;
  int cus = 0;
  int rc = device_cus(&cus);
  if (rc) return rc;
  const int64_t qtiles = (a.nq + fBQ - 1) / fBQ;
  int64_t bx = (int64_t)cus * FX_I3_BPC;  // workgroups per CU
  if (bx > a.num_tiles * kI3Sub) bx = a.num_tiles * kI3Sub;
  for (int64_t y0 = 0; y0 < qtiles; y0 += 65535) {
    FilterArgs b = a;
    const int64_t yn = (qtiles - y0) < 65535 ? (qtiles - y0) : 65535;
    b.Qh = a.Qh + y0 * fBQ * 32;  // (64 B per query and chunk in both formats)
    b.qinfo = a.qinfo + y0 * fBQ * (a.img8 ? kI8QInfo : 4);
    b.thr = a.thr + y0 * fBQ;
    b.count = a.count + y0 * fBQ * kCountStride;
    b.cand = a.cand + y0 * fBQ * (int64_t)a.cap;
    if (a.cand_ub) b.cand_ub = a.cand_ub + y0 * fBQ * (int64_t)a.cap;
    b.nq = a.nq - y0 * fBQ;
    void* args[] = {(void*)&b};
    hipError_t e = hipLaunchKernel(fn, dim3((unsigned)bx, (unsigned)yn), dim3(kI3Threads), args,
                                   smem, stream);
    if (e != hipSuccess) {
      set_error("filter_img3_kernel launch: %s", hipGetErrorString(e));
      return FX_EHIP;
    }
  }
  return check_launch("filter_img3_kernel");
}

#if FX_FILTER_BQ >= 256
// ---- int8 image, the queries held in registers (filter_img8_kernel)
//
// filter_img3_kernel keeps each wave's image rows in registers and streams
// the 256-query tile through LDS: every 64-component chunk of every 256-row
// tile DMAs the queries again from L2, as many bytes as the image itself
// (without those DMAs the final pass ran 25 % faster).  Here
// the operands swap roles: wave w holds queries 32 w .. 32 w + 31 as MFMA A
// operands for every k-step (24 x 16 B per lane: d <= 768) for the whole
// kernel, and the image goes through a 4-slot LDS ring by DMA straight from
// HBM (16 KB chunks: 128 rows x 4 k-steps, each 32-row k-step one contiguous
// KB in the image's fragment order, read back as the B operand with one
// conflict-free ds_read_b128).  The only bytes that move are the image's,
// once.  The accumulator of a (32-query, 32-row) tile then holds one row per
// lane and 16 queries: the pass test is i8_epilogue's with the pairs taken
// over queries instead of rows (the same f32 operations per (row, query)
// pair: bit-identical decisions), appends one LDS atomic per passing pair.
// Serves 256-query batches (not all-pass) of int8 images with d <= 768.
#ifndef FX_I8T
#define FX_I8T 1
#endif
#ifndef FX_T8_SLOTS
#define FX_T8_SLOTS 4  // ring slots of 16 KB (FX_T8_SLOTS - 1 chunks in flight)
#endif
#ifndef FX_T8_SEG
#define FX_T8_SEG 40   // LDS append entries per query (8 B each; past them: global slots)
#endif
#ifndef FX_T8_PAIR
#define FX_T8_PAIR 1   // 1: the ring refilled two chunks at a time, one barrier per two
                       // chunks (an even chunk count per tile; FX_T8_SLOTS even)
#endif
#ifndef FX_T8_PRIO
#define FX_T8_PRIO 0   // 1: waves 4-7 (each SIMD's second wave) at s_setprio 1
#endif
constexpr int kT8Waves = 8;
constexpr int kT8Threads = 64 * kT8Waves;
constexpr int kT8BM = 128;                            // rows per workgroup tile
constexpr int kT8RT = kT8BM / 32;                     // 32-row tiles (B operands)
constexpr int kT8Sub = fBM / kT8BM;                   // workgroup tiles per plan tile
constexpr int kT8KS = 24;                             // k-steps in registers (d <= 768)
constexpr int kT8CK = 4;                              // k-steps per ring chunk
constexpr int kT8NC = kT8KS / kT8CK;                  // ring chunks per tile, at most
constexpr int kT8SlotBytes = kT8RT * kT8CK * 1024;    // 16 KB
constexpr int kT8Slots = FX_T8_SLOTS;
constexpr int kT8QA = kT8Slots - 1;                   // chunks in flight
constexpr int kT8Dma = kT8SlotBytes / 1024 / kT8Waves;  // 1-KB DMAs per wave per chunk
constexpr int kT8SEG = FX_T8_SEG;
constexpr int kT8Hi = kT8SEG * 3 / 4;  // a segment this full asks for a flush
static_assert(kT8Waves * 32 == fBQ && kT8Sub * kT8BM == fBM && kT8Dma == 2 &&
                  kT8RT * kT8CK == kT8Waves * kT8Dma,
              "filter_img8_kernel tiling");
struct Img8Shared {
  unsigned char ring[kT8Slots][kT8SlotBytes];
  float rinfo[kT8BM];   // omega (NaN: forced)
  float rterm[kT8BM];   // y1
  float rext[kT8BM];    // 1 / s
  uint32_t rrow[kT8BM];   // the global corpus row (image8_perm)
  uint32_t rkeep[kT8BM];  // 1: a row in range and not masked out
  f32x4 qtab[fBQ];
  f32x4 qinf[fBQ];
  uint32_t segc[fBQ];     // appends per query since the last flush (past kT8SEG: global)
  uint32_t segn[fBQ];     // (flush) entries of the query's segment
  uint32_t segbase[fBQ];  // (flush) their first candidate slot
  uint32_t flush;         // a segment passed kT8Hi: flush at the next tile start
  uint2 sege[fBQ * kT8SEG];  // entries {accumulator bits, image row}; bounds at the flush
};
static_assert(sizeof(Img8Shared) <= 160 * 1024, "filter_img8_kernel: LDS over 160 KB");

// Pass test and appends of one wave's (32 queries x 128 rows) accumulators:
// acc[t] element j is row 32 t + l32 against query 32 wid + (j & 3) + 8 (j >> 2) + 4 h.
template <int METRIC, bool ALL>
__device__ __forceinline__ void t8_epilogue(const f32x16 (&acc)[kT8RT], Img8Shared* sh,
                                            const FilterArgs& a, int64_t q0, int64_t r0, int64_t ti,
                                            int wid, int h, int l32) {
  constexpr int SEG = kT8SEG;
  float om[kT8RT], y1[kT8RT], y2[kT8RT];
  uint32_t keep[kT8RT];
#pragma unroll
  for (int t = 0; t < kT8RT; ++t) {
    const int lr = t * 32 + l32;
    om[t] = sh->rinfo[lr];
    y1[t] = sh->rterm[lr];
    y2[t] = METRIC == 0 ? sh->rext[lr] : 0.f;
    keep[t] = sh->rkeep[lr] ? 0xffffu : 0u;
  }
  const int qb = wid * 32 + 4 * h;  // query of element j: qb + (j & 3) + 8 (j >> 2)
  if constexpr (ALL) {
    // a sampling phase's first launch (upper bounds only, then the k-th
    // smallest): every pair, at a fixed slot -- tile ti's row lr at ti * 128
    // + lr (the plan keeps the phase within cap), an empty key for a row
    // that is masked out or past the end; the counts are set by workgroup 0
    // (the element loop rolled, its accumulator picked by a select tree:
    // 64 unrolled bounds spilled)
    auto pick = [](float lo, float hi, uint32_t m) {
      return __uint_as_float((__float_as_uint(hi) & m) | (__float_as_uint(lo) & ~m));
    };
#pragma unroll
    for (int t = 0; t < kT8RT; ++t) {
      const int lr = t * 32 + l32;
      const uint32_t grow = sh->rrow[lr];
      const float ys = sh->rext[lr];
      const size_t p = (size_t)ti * kT8BM + lr;
#pragma unroll 1
      for (int j = 0; j < 16; ++j) {
        const int qi = qb + (j & 3) + 8 * (j >> 2);
        const int64_t gq = q0 + qi;
        if (gq >= a.nq) continue;
        const uint32_t m0 = 0u - ((uint32_t)j & 1u), m1 = 0u - (((uint32_t)j >> 1) & 1u);
        const uint32_t m2 = 0u - (((uint32_t)j >> 2) & 1u), m3 = 0u - (((uint32_t)j >> 3) & 1u);
        float v8[8], v4[4], v2[2];
#pragma unroll
        for (int i = 0; i < 8; ++i) v8[i] = pick(acc[t][2 * i], acc[t][2 * i + 1], m0);
#pragma unroll
        for (int i = 0; i < 4; ++i) v4[i] = pick(v8[2 * i], v8[2 * i + 1], m1);
#pragma unroll
        for (int i = 0; i < 2; ++i) v2[i] = pick(v4[2 * i], v4[2 * i + 1], m2);
        float lb, ub;
        i8_bounds<METRIC>(pick(v2[0], v2[1], m3), om[t], y1[t], ys, sh->qinf[qi], a.d, lb, ub);
        __builtin_nontemporal_store(keep[t] ? make_comp(ub, grow) : kEmpty,
                                    a.cand + (size_t)gq * a.cap + p);
      }
    }
    return;
  }
  uint32_t qlive = 0u;
#pragma unroll
  for (int j = 0; j < 16; ++j)
    qlive |= (q0 + qb + (j & 3) + 8 * (j >> 2) < a.nq ? 1u : 0u) << j;
  // fail bit j enters last-in at bit 0: pairs (j, j + 1) run down
  uint32_t fail[kT8RT];
#pragma unroll
  for (int t = 0; t < kT8RT; ++t) fail[t] = 0u;
  const f32x2 nc0 = {-kI8C0, -kI8C0};
#pragma unroll
  for (int jp = 7; jp >= 0; --jp) {
    const int j = 2 * jp;
    const int q = qb + (j & 3) + 8 * (j >> 2);  // queries q, q + 1
    const f32x4 ca = sh->qtab[q], cb = sh->qtab[q + 1];
    const f32x2 ra = {ca[0], cb[0]}, c1 = {ca[1], cb[1]}, c2 = {ca[2], cb[2]};
#pragma unroll
    for (int t = 0; t < kT8RT; ++t) {
      const f32x2 xp = {acc[t][j], acc[t][j + 1]};
      f32x2 v = __builtin_elementwise_fma(f32x2{om[t], om[t]}, ra, xp);
      v = __builtin_elementwise_fma(f32x2{y1[t], y1[t]}, c1, v);
      if constexpr (METRIC == 0) v = __builtin_elementwise_fma(f32x2{y2[t], y2[t]}, c2, v);
      const f32x2 dd = v + nc0;
      fail[t] = __builtin_amdgcn_alignbit(fail[t], __float_as_uint(dd[1]), 31);
      fail[t] = __builtin_amdgcn_alignbit(fail[t], __float_as_uint(dd[0]), 31);
    }
  }
  uint32_t pm[kT8RT], any = 0u;
#pragma unroll
  for (int t = 0; t < kT8RT; ++t) {
    const uint32_t force = om[t] != om[t] ? ~0u : 0u;  // a forced row passes every query
    pm[t] = (~fail[t] | force) & keep[t] & qlive;
    any |= pm[t];
  }
  if (__ballot(any != 0u) == 0ull) return;
#ifdef FX_T8_DIAG  // 4: the pass test without its appends (the final pass only)
  if ((FX_T8_DIAG & 4) && a.skip_full) {
    if (any == 0x12345u) a.count[0] = 7;
    return;
  }
#endif
  // appends: the accumulator bits and the image row into the query's LDS
  // segment (8 B; the bounds are computed at the flush, t8_flush); past the
  // segment (rare: the flush keeps it under kT8Hi between tiles) a global
  // slot with the bounds computed here
  static_for<kT8RT>([&](auto tc) {
    constexpr int t = decltype(tc)::value;
    uint32_t bits = pm[t];
    if (__ballot(bits != 0u) == 0ull) return;
    const int lr = t * 32 + (int)opaque((unsigned)l32);
    const uint32_t irow = (uint32_t)(r0 + lr);
    while (bits != 0u) {
      const int j = __builtin_ctz(bits);
      bits &= bits - 1u;
      auto pick = [](float lo, float hi, uint32_t m) {
        return __uint_as_float((__float_as_uint(hi) & m) | (__float_as_uint(lo) & ~m));
      };
      const uint32_t m0 = 0u - ((uint32_t)j & 1u), m1 = 0u - (((uint32_t)j >> 1) & 1u);
      const uint32_t m2 = 0u - (((uint32_t)j >> 2) & 1u), m3 = 0u - (((uint32_t)j >> 3) & 1u);
      float v8[8], v4[4], v2[2];
#pragma unroll
      for (int i = 0; i < 8; ++i) v8[i] = pick(acc[t][2 * i], acc[t][2 * i + 1], m0);
#pragma unroll
      for (int i = 0; i < 4; ++i) v4[i] = pick(v8[2 * i], v8[2 * i + 1], m1);
#pragma unroll
      for (int i = 0; i < 2; ++i) v2[i] = pick(v4[2 * i], v4[2 * i + 1], m2);
      const float x = pick(v2[0], v2[1], m3);
      const int qi = qb + (j & 3) + 8 * (j >> 2);
#ifdef FX_T8_DIAG  // (timing builds, the final pass only: 8 no LDS atomic, 16 no entry
                   // write, 32 neither; its flush writes nothing)
      uint32_t p;
      if ((FX_T8_DIAG & 40) && a.skip_full)
        p = (uint32_t)j & 15u;
      else
        p = lds_add_rtn_u32(&sh->segc[qi], 1u);
      if ((FX_T8_DIAG & 48) && a.skip_full) {
        if (__float_as_uint(x) == 0x12345u && p == 3u) a.count[0] = irow;
        continue;
      }
#else
      const uint32_t p = lds_add_rtn_u32(&sh->segc[qi], 1u);
#endif
      if (p < (uint32_t)SEG) {
        lds_write2_u32(&sh->sege[qi * SEG + p], __float_as_uint(x), irow);
        if (p == (uint32_t)kT8Hi) lds_write1_u32(&sh->flush, 1u);
      } else {
        const int64_t gq = q0 + qi;
        float lb, ub;
        i8_bounds<METRIC>(x, om[t], y1[t], sh->rext[lr], sh->qinf[qi], a.d, lb, ub);
        const uint32_t grow = sh->rrow[lr];
        const uint32_t gp = atomicAdd(&a.count[gq * kCountStride], 1u);
        if (gp < (uint32_t)a.cap) {
          const size_t slot = (size_t)gq * a.cap + gp;
          if (a.cand_ub != nullptr) {
            a.cand[slot] = make_comp(lb, grow);
            a.cand_ub[slot] = make_comp(ub, grow);
          } else {
            a.cand[slot] = make_comp(ub, grow);
          }
        }
      }
    }
  });
}

// Write the segments out (every thread; between two barriers of the tile
// loop, or at the end): one global atomic per query reserves the slots, the
// entries get their bounds from the row's terms (a.rowinfo) and the query's
// record; RESET empties the segments for the next tiles.
template <int METRIC, bool RESET>
__device__ __forceinline__ void t8_flush(Img8Shared* sh, const FilterArgs& a, int64_t q0, int tid) {
  constexpr int SEG = kT8SEG;
#ifdef FX_T8_DIAG
  if ((FX_T8_DIAG & 56) && a.skip_full) {  // (entries not written: nothing to flush)
    __syncthreads();
    for (int q = tid; q < fBQ; q += kT8Threads) sh->segc[q] = 0u;
    if (tid == 0) sh->flush = 0u;
    return;
  }
#endif
  for (int q = tid; q < fBQ; q += kT8Threads) {
    const uint32_t n = sh->segc[q] < (uint32_t)SEG ? sh->segc[q] : (uint32_t)SEG;
    sh->segn[q] = n;
    sh->segbase[q] = n != 0u && q0 + q < a.nq ? atomicAdd(&a.count[(q0 + q) * kCountStride], n) : 0u;
  }
  __syncthreads();
  for (int i = tid; i < fBQ * SEG; i += kT8Threads) {
    const int q = i / SEG, j = i % SEG;
    if ((uint32_t)j >= sh->segn[q]) continue;
    const uint32_t p = sh->segbase[q] + (uint32_t)j;
    if (p >= (uint32_t)a.cap) continue;
    const uint2 e = sh->sege[i];
    const int64_t row = (int64_t)e.y;
    const f32x4 ri = *reinterpret_cast<const f32x4*>(a.rowinfo + row * kI8RowInfo);
    const float y1 = METRIC == 1 ? ri[1] : METRIC == 2 ? ri[2] : ri[3];
    float lb, ub;
    i8_bounds<METRIC>(__uint_as_float(e.x), ri[0], y1, ri[1], sh->qinf[q], a.d, lb, ub);
    const uint32_t grow = (uint32_t)a.row_base + perm_row(a.perm_a, a.n, row);
    const size_t slot = (size_t)(q0 + q) * a.cap + p;
    if (a.cand_ub != nullptr) {
      a.cand[slot] = make_comp(lb, grow);
      a.cand_ub[slot] = make_comp(ub, grow);
    } else {
      a.cand[slot] = make_comp(ub, grow);
    }
  }
  if constexpr (RESET) {
    __syncthreads();  // (every entry read)
    for (int q = tid; q < fBQ; q += kT8Threads) sh->segc[q] = 0u;
    if (tid == 0) sh->flush = 0u;
    // (the next appends follow the tile's epilogue barrier)
  }
}

// NCH: ring chunks per tile, ceil(ceil(d / 32) / 4) (a compile-time chunk
// loop: straight-line code, where the compiler counts every wait exactly)
// ALL: an all-pass sampling launch (t8_epilogue; its own instantiation, whose
// unrolled bounds would otherwise spill the pass-test kernel's registers)
template <int METRIC, int NCH, bool ALL>
__global__ void __launch_bounds__(kT8Threads, 2) filter_img8_kernel(FilterArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  Img8Shared* sh = reinterpret_cast<Img8Shared*>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, l32 = lane & 31;
  const int64_t q0 = (int64_t)blockIdx.y * fBQ;
  const int ksteps = (a.d + 31) / 32;  // the image's k-steps per 32-row tile (<= 4 NCH)
  constexpr int nch = NCH;
  static_assert(NCH >= 1 && NCH <= kT8NC, "filter_img8_kernel: d <= 768");
  const int64_t ntile32 = (a.n + 31) / 32;
  const int64_t ntiles = a.num_tiles * kT8Sub;
  auto tile_r0 = [&](int64_t ti) {
    return (a.tile_start + (ti / kT8Sub) * a.tile_stride) * fBM + (ti % kT8Sub) * kT8BM;
  };
  if ((int64_t)blockIdx.x >= ntiles) return;
  if (a.skip_full) {  // every query of the tile predicted to overflow: nothing to do
    bool full = true;
    for (int q = tid; q < fBQ; q += kT8Threads)
      if (q0 + q < a.nq && a.count[(q0 + q) * kCountStride] <= (uint32_t)a.cap) full = false;
    if (__syncthreads_and(full)) return;
  }
  i8_query_table<METRIC>(a, q0, sh->qtab, sh->qinf, tid, kT8Threads);
  for (int q = tid; q < fBQ; q += kT8Threads) sh->segc[q] = 0u;
  if (ALL && blockIdx.x == 0)  // every slot of the phase (t8_epilogue)
    for (int q = tid; q < fBQ; q += kT8Threads)
      if (q0 + q < a.nq) a.count[(q0 + q) * kCountStride] = (uint32_t)(ntiles * kT8BM);
  if (tid == 0) sh->flush = 0u;
  // the wave's 32 queries, every k-step: chunk c of query q is 64 B at
  // (c * qstride + q) * 64 (qprep8), k-step s its half s & 1 (zeros past dq)
  i32x4 qa[kT8KS];
  {
    const unsigned char* qb = reinterpret_cast<const unsigned char*>(a.Qh + q0 * 32);
    const int qchunks = a.dq / 64;
    const int64_t qo = (int64_t)(wid * 32 + l32) * 64 + h * 16;
#pragma unroll
    for (int s = 0; s < kT8KS; ++s) {
      const int c = s >> 1;
      qa[s] = c < qchunks ? *reinterpret_cast<const i32x4*>(qb + (int64_t)c * a.qstride * 64 + qo +
                                                             (s & 1) * 32)
                          : i32x4(0);
    }
  }
  __syncthreads();

  // the ring: chunk c of a tile holds its 4 32-row tiles x k-steps 4 c .. 4 c
  // + 3, KB (tt, kk) at (4 tt + kk) KB; wave w DMAs tile tt = w / 2, k-steps
  // 2 (w & 1), + 1 (past ksteps: dropped, the slot keeps an earlier chunk's
  // finite bytes, multiplied by zero query k-steps; past the rows: an empty
  // descriptor, rows the epilogue skips)
  const int tt = wid >> 1, kk0 = (wid & 1) * 2;
  auto x_rsrc = [&](int64_t ti) {
    const int64_t t32 = tile_r0(ti) / 32 + tt;
    const int64_t live = (ti < ntiles && t32 < ntile32) ? 1 : 0;
    const unsigned char* base = reinterpret_cast<const unsigned char*>(a.X) +
                                (live ? t32 : 0) * (int64_t)ksteps * 1024;
    const uint64_t xp = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)xp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(xp >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)(live * ksteps * 1024));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                             nb, 0x00020000);
  };
  const uint32_t xl = (uint32_t)opaque((unsigned)lane) * 16u;
  int64_t xt = blockIdx.x;  // tile and chunk of the next DMA
  int xc = 0, wslot = 0;
  __amdgpu_buffer_rsrc_t xr = x_rsrc(xt);
  auto issue = [&]() {
    unsigned char* st = sh->ring[wslot] + (tt * kT8CK + kk0) * 1024;
#pragma unroll
    for (int i = 0; i < kT8Dma; ++i) {
      const int s = xc * kT8CK + kk0 + i;  // (wave-uniform)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (i3_lds_ptr)(st + i * 1024), 16,
                                               s < ksteps ? xl : 0x7fff0000u, s * 1024, 0, 0);
    }
    if (++xc == nch) {
      xc = 0;
      xt += gridDim.x;
      xr = x_rsrc(xt);
    }
    wslot = wslot + 1 == kT8Slots ? 0 : wslot + 1;
  };
  // (pairs: the ring holds kT8Slots / 2 pairs, all but one in flight)
  constexpr bool PAIR = FX_T8_PAIR && NCH % 2 == 0;
  static_assert(!FX_T8_PAIR || kT8Slots % 2 == 0, "FX_T8_PAIR: an even ring");
  constexpr int kAhead = PAIR ? kT8Slots - 2 : kT8QA;  // chunks issued ahead of the one read
#pragma unroll
  for (int i = 0; i < kAhead; ++i) issue();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (once: the query fragments too)

  f32x16 acc[kT8RT];
  const f32x16 acc0 = f32x16(kI8Magic);  // see "int8 filter image"
  int rslot = 0;
  if (FX_T8_PRIO && wid >= 4) __builtin_amdgcn_s_setprio(1);
  const int lr = tid & (kT8BM - 1);  // the row this thread notes (threads >= kT8BM: duplicates)
  for (int64_t ti = blockIdx.x; ti < ntiles; ti += gridDim.x) {
    const int64_t r0 = tile_r0(ti);
    f32x4 rsum = {};
    uint32_t mword = ~0u;  // (no mask: every row)
    static_for<NCH>([&](auto cc) {
      constexpr int C = decltype(cc)::value;
      // chunk C landed: after its DMAs this wave issued QA - 1 chunks' DMAs
      // (and possibly the rows' terms: a stronger wait), and every wave is
      // done with the slot refilled next
      if constexpr (PAIR) {
        // even chunks only: the pair (C, C + 1) landed (after its DMAs this
        // wave issued the kAhead / 2 - 1 pairs ahead of it), every wave done
        // with the pair refilled next
        if constexpr (C % 2 == 0) {
          i3_wait_barrier<(kAhead - 2) * kT8Dma>();
          issue();
          issue();
        }
      } else {
        i3_wait_barrier<(kT8QA - 1) * kT8Dma>();
        issue();
      }
      // (after the tile's first barrier every wave is past the last
      // epilogue: a segment that passed kT8Hi is written out now)
      if constexpr (C == 0) {
        if (sh->flush) t8_flush<METRIC, true>(sh, a, q0, tid);
      }
      if constexpr (C == 0) {  // the rows' terms and mask words of this tile
        const int64_t row = r0 + lr < a.n ? r0 + lr : a.n - 1;
        rsum = *reinterpret_cast<const f32x4*>(a.rowinfo + row * kI8RowInfo);
        // (used at the tile's last chunk; no load without a mask: a load of
        // the row's terms there was merged with rsum's, and waited for here)
        if (a.mask != nullptr) mword = a.mask[perm_row(a.perm_a, a.n, row) >> 5];
      }
      // the k-steps of this barrier interval (chunks C .. C + G - 1) in one
      // stream, B fragments read two k-steps ahead: k-step j + 2's reads
      // issue before k-step j's MFMAs, across the pair's chunk boundary too
      constexpr int G = PAIR ? 2 : 1;
      if constexpr (C % G == 0) {
        constexpr int J = G * kT8CK;
        typedef int i32x16 __attribute__((ext_vector_type(16)));
        auto read_b = [&](i32x4 (&b)[kT8RT], auto jc) {
          constexpr int j = decltype(jc)::value;
          const int slot = rslot + j / kT8CK < kT8Slots ? rslot + j / kT8CK : rslot + j / kT8CK - kT8Slots;
          const unsigned char* st = sh->ring[slot] + lane * 16 + (j % kT8CK) * 1024;
#pragma unroll
          for (int t = 0; t < kT8RT; ++t) b[t] = *reinterpret_cast<const i32x4*>(st + t * kT8CK * 1024);
        };
        auto mfma4 = [&](const i32x4 (&b)[kT8RT], auto jc) {
          constexpr int j = decltype(jc)::value;
          constexpr int s = (C + j / kT8CK) * kT8CK + j % kT8CK;  // the query k-step
#pragma unroll
          for (int t = 0; t < kT8RT; ++t) {
#ifdef FX_T8_DIAG  // 2: no MFMA in the final pass (the B reads stay live)
            if ((FX_T8_DIAG & 2) && a.skip_full) {
              if (s == 0) acc[t] = acc0;
              acc[t][0] += __builtin_bit_cast(float, b[t][0] ^ qa[s][0]);
              continue;
            }
#endif
            const f32x16 cin = s == 0 ? acc0 : acc[t];
            acc[t] = __builtin_bit_cast(
                f32x16, __builtin_amdgcn_mfma_i32_32x32x32_i8(qa[s], b[t],
                                                              __builtin_bit_cast(i32x16, cin), 0, 0, 0));
          }
        };
        i32x4 b0[kT8RT], b1[kT8RT];
        read_b(b0, std::integral_constant<int, 0>{});
        read_b(b1, std::integral_constant<int, 1>{});
        __builtin_amdgcn_sched_barrier(0);
        static_for<J>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          if constexpr (j % 2 == 0)
            mfma4(b0, jc);
          else
            mfma4(b1, jc);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (j + 2 < J) {
            if constexpr (j % 2 == 0)
              read_b(b0, std::integral_constant<int, j + 2>{});
            else
              read_b(b1, std::integral_constant<int, j + 2>{});
            __builtin_amdgcn_sched_barrier(0);
          }
        });
        rslot = rslot + G < kT8Slots ? rslot + G : rslot + G - kT8Slots;
      }
      // one thread per row notes its terms for the epilogue, after the last
      // chunk's MFMAs: in this unrolled straight line the compiler counts
      // the exact wait for the terms' loads (landed by now: they retire
      // before the chunk waits of steps 3 on), where after the loop it
      // could only wait vmcnt(0), for the next tile's DMAs too (the rows of
      // the previous tile's epilogue were read before this tile's first barrier)
      if (C == NCH - 1 && tid < kT8BM) {
        const int lr = (int)opaque((unsigned)tid);
        const int64_t row = r0 + lr;
        const int64_t mrow = perm_row(a.perm_a, a.n, row < a.n ? row : a.n - 1);
        const bool ok = row < a.n && ((mword >> (mrow & 31)) & 1u);
        // (every lane of the terms' load stays live to here: a dead one was
        // reused for the mask word, whose write then waited for the load)
        asm volatile("" ::"v"(rsum[0]), "v"(rsum[1]), "v"(rsum[2]), "v"(rsum[3]));
        sh->rinfo[lr] = rsum[0];
        sh->rterm[lr] = METRIC == 1 ? rsum[1] : METRIC == 2 ? rsum[2] : rsum[3];
        sh->rext[lr] = rsum[1];
        sh->rrow[lr] = (uint32_t)a.row_base + (row < a.n ? (uint32_t)mrow : 0u);
        sh->rkeep[lr] = ok ? 1u : 0u;
      }
    });
    // (the barrier also separates the tile's last MFMAs from the epilogue's
    // reads of their accumulators)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#ifdef FX_T8_DIAG  // (timing builds only: 1 no epilogue in the final pass)
    if ((FX_T8_DIAG & 1) && a.skip_full) {
      if (acc[0][0] == 1.2345f && acc[3][15] == 2.f) a.count[0] = 7;
      continue;
    }
#endif
    t8_epilogue<METRIC, ALL>(acc, sh, a, q0, r0, ti, wid, h, l32);
  }
  // the ring's last DMAs (past the end) land before the workgroup's LDS is
  // released; then the segments go out
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  t8_flush<METRIC, false>(sh, a, q0, tid);
}

static bool img8_serves(const FilterArgs& a) {
  // (an all-pass launch with both bounds -- a one-phase plan's F1 -- stays
  // with the appending kernels; a sampling phase's slots fit: the plan keeps
  // its rows within cap)
  return FX_I8T && a.img8 && (!a.all_pass || (a.cand_ub == nullptr &&
                                               a.num_tiles * fBM <= (int64_t)a.cap)) &&
         a.dq <= kT8KS * 32 && (a.d + 31) / 32 <= kT8KS && option(kOptImg8) != 0;
}

template <int NCH, bool ALL>
static const void* img8_fn_all(int metric) {
  return metric == FX_METRIC_COS  ? (const void*)filter_img8_kernel<2, NCH, ALL>
         : metric == FX_METRIC_IP ? (const void*)filter_img8_kernel<1, NCH, ALL>
                                  : (const void*)filter_img8_kernel<0, NCH, ALL>;
}
template <int NCH>
static const void* img8_fn(int metric, bool all) {
  return all ? img8_fn_all<NCH, true>(metric) : img8_fn_all<NCH, false>(metric);
}

static int launch_img8(const FilterArgs& a, int metric, hipStream_t stream) {
  const size_t smem = sizeof(Img8Shared);
  const int nch = ((a.d + 31) / 32 + kT8CK - 1) / kT8CK;
  const bool all = a.all_pass != 0;
  const void* fn = nch <= 1   ? img8_fn<1>(metric, all)
                   : nch == 2 ? img8_fn<2>(metric, all)
                   : nch == 3 ? img8_fn<3>(metric, all)
                   : nch == 4 ? img8_fn<4>(metric, all)
                   : nch == 5 ? img8_fn<5>(metric, all)
                              : img8_fn<6>(metric, all);
  if (int rc = allow_lds(fn)) return rc;
  int cus = 0;
  int rc = device_cus(&cus);
  if (rc) return rc;
  const int64_t qtiles = (a.nq + fBQ - 1) / fBQ;
  int64_t bx = (int64_t)cus;  // one workgroup per CU (its LDS)
  if (bx > a.num_tiles * kT8Sub) bx = a.num_tiles * kT8Sub;
  for (int64_t y0 = 0; y0 < qtiles; y0 += 65535) {
    FilterArgs b = a;
    const int64_t yn = (qtiles - y0) < 65535 ? (qtiles - y0) : 65535;
    b.Qh = a.Qh + y0 * fBQ * 32;
    b.qinfo = a.qinfo + y0 * fBQ * kI8QInfo;
    b.thr = a.thr + y0 * fBQ;
    b.count = a.count + y0 * fBQ * kCountStride;
    b.cand = a.cand + y0 * fBQ * (int64_t)a.cap;
    if (a.cand_ub) b.cand_ub = a.cand_ub + y0 * fBQ * (int64_t)a.cap;
    b.nq = a.nq - y0 * fBQ;
    void* args[] = {(void*)&b};
    hipError_t e = hipLaunchKernel(fn, dim3((unsigned)bx, (unsigned)yn), dim3(kT8Threads), args,
                                   smem, stream);
    if (e != hipSuccess) {
      set_error("filter_img8_kernel launch: %s", hipGetErrorString(e));
      return FX_EHIP;
    }
  }
  return check_launch("filter_img8_kernel");
}
#endif  // FX_FILTER_BQ >= 256

#if FX_FILTER_BQ <= 128
// ---- int8 image, a resident query slice (filter_img6_kernel)
//
// filter_img3_kernel streams the query tile through an LDS ring: every
// 64-component chunk of every 256-row tile DMAs the tile's queries again
// (as many bytes per chunk as the image itself) behind a workgroup barrier,
// so the 8 waves run in lockstep and the MFMAs add to the image stream
// instead of hiding under it.  Here a workgroup holds its
// slice of 128 queries (the q128 build; 64 in q64i) in LDS for the whole
// kernel (96 KB at 768-d, XOR-swizzled for conflict-free ds_read_b128) and
// each of its waves runs its own 32-row tiles with FX_I6_XS image k-steps in
// flight in registers across tile ends, its own rows' terms and flags in
// LDS, and the same epilogue (i8_epilogue: pass test, bounds, LDS append
// segments shared through LDS atomics); the only barrier of the tile loop
// is the one before the epilogue (see there).  Default for batches of up to
// 128 queries (launch_filter).  With option img6 = 2 a larger batch runs its
// slices on different CUs over the same tiles at the same time --
// workgroup (x, y) takes slice y and tiles x, x + G, ... with G = CUs /
// slices, so the partners share an XCD (x + G y = x mod 8) and the second
// read of a tile can come from its L2 or the Infinity Cache; measured slower
// than filter_img3_kernel's 256-query tiles (3.34 vs 2.97 ms), so off.
#ifndef FX_I6_XS
#define FX_I6_XS 8
#endif
constexpr int kI6Waves = 8;
constexpr int kI6Threads = 64 * kI6Waves;
constexpr int kI6BM = 32 * kI6Waves;
static_assert(kI6BM == fBM, "one plan tile per workgroup tile");
constexpr int kI6SEG = FX_I3_SEG;
constexpr int kI6SliceBatch = 12;  // 768-d, 128 queries: every piece of the slice in one batch
struct Img6Shared {
  float rinfo[kI6BM];
  float rterm[kI6BM];
  float rext[kI6BM];
  uint32_t rrow[kI6BM];
  uint32_t rflags[kRowFlagWords];
  f32x4 qtab[fBQ];
  f32x4 qinf[fBQ];
  uint32_t seg[fBQ + 3 * fBQ * kI6SEG];
  uint32_t segbase[fBQ];
};
// the query slice follows: (dq / 64) chunks x 128 queries x 64 B
static size_t img6_smem(int dq) { return sizeof(Img6Shared) + (size_t)(dq / 64) * fBQ * 64; }
bool img6_fits(int dq) { return img6_smem(dq) <= 160 * 1024; }

template <int METRIC>
__global__ void __launch_bounds__(kI6Threads, 1) filter_img6_kernel(FilterArgs a) {
  constexpr int XS = FX_I6_XS, SEG = kI6SEG;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  Img6Shared* sh = reinterpret_cast<Img6Shared*>(smem);
  unsigned char* qslice = smem + sizeof(Img6Shared);
#ifdef FX_DIAG_BUILD
  const int diag = a.diag;
#else
  constexpr int diag = 0;
#endif
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, l32 = lane & 31;
  const int64_t q0 = (int64_t)blockIdx.y * fBQ;
  const int ksteps = (a.d + 31) / 32;
  const int nks = (ksteps + XS - 1) / XS * XS;  // (past the row end the image reads zeros)
  const int ngroups = nks / XS;
  const int64_t ntile32 = (a.n + 31) / 32;
  const int64_t ntiles = a.num_tiles;
  if ((int64_t)blockIdx.x >= ntiles) return;
  if (a.skip_full) {  // every query of the slice predicted to overflow (the gate): the
                      // exact scan recomputes them, so the final pass has nothing to do
    bool full = true;
    for (int q = tid; q < fBQ; q += kI6Threads)
      if (q0 + q < a.nq && a.count[(q0 + q) * kCountStride] <= (uint32_t)a.cap) full = false;
    if (__syncthreads_and(full)) return;
  }
  i8_query_table<METRIC>(a, q0, sh->qtab, sh->qinf, tid, kI6Threads);
  for (int q = tid; q < fBQ; q += kI6Threads) sh->seg[q] = 0u;
  // the slice's live queries share all fBQ * SEG segment entries (one query:
  // 1 536 instead of 24, so a k = 1 000 search's ~200 appends per workgroup
  // and phase stay in LDS instead of each lane taking a slot from the one
  // global counter of the query: F1 429 us at 6.25M x 1536)
  const int64_t nlive = a.nq - q0 < fBQ ? a.nq - q0 : fBQ;
  const int segcap = (fBQ * SEG) / (int)(nlive > 0 ? nlive : 1);
  {  // the slice: chunk c of query Q at (c * 128 + Q) * 64, piece p at (p ^ ((Q >> 2) & 3)) * 16
    // (kI6SliceBatch loads in flight per thread before their stores: one
    // load, wait, store per iteration cost ~1.5 us each, ~18 us per launch)
    const int total = a.dq / 64 * fBQ * 4;
    const unsigned char* qb = reinterpret_cast<const unsigned char*>(a.Qh);
    for (int i0 = tid; i0 < total; i0 += kI6SliceBatch * kI6Threads) {
      i32x4 v[kI6SliceBatch];
#pragma unroll
      for (int j = 0; j < kI6SliceBatch; ++j) {
        const int i = i0 + j * kI6Threads;
        const int c = i / (fBQ * 4), Q = (i / 4) % fBQ, pc = i % 4;
        if (i < total)
          v[j] = *reinterpret_cast<const i32x4*>(qb + ((int64_t)c * a.qstride + q0 + Q) * 64 +
                                                 pc * 16);
      }
#pragma unroll
      for (int j = 0; j < kI6SliceBatch; ++j) {
        const int i = i0 + j * kI6Threads;
        const int c = i / (fBQ * 4), Q = (i / 4) % fBQ, pc = i % 4;
        if (i < total)
          *reinterpret_cast<i32x4*>(qslice + ((c * fBQ + Q) * 64 + ((pc ^ ((Q >> 2) & 3)) * 16))) =
              v[j];
      }
    }
  }
  __syncthreads();
  // B fragment of query tile u at k-step ks: query Q = 32 u + l32, piece
  // 2 (ks & 1) + h of chunk ks / 2 (bits 2-3 of Q do not depend on u)
  const int bsw = (l32 >> 2) & 3;
  auto bfrag = [&](int ks, int u) {
    const int Q = 32 * u + l32;
    return *reinterpret_cast<const f16x8*>(
        qslice + ((ks >> 1) * fBQ + Q) * 64 + (((2 * (ks & 1) + h) ^ bsw) * 16));
  };
  auto tile_r0 = [&](int64_t ti) { return (a.tile_start + ti * a.tile_stride) * fBM; };
  auto x_rsrc = [&](int64_t ti) {
    const int64_t t32 = tile_r0(ti) / 32 + wid;
    const int64_t live = (ti < ntiles && t32 < ntile32) ? 1 : 0;
    const unsigned char* base = reinterpret_cast<const unsigned char*>(a.X) +
                                (live ? t32 : 0) * (int64_t)ksteps * 1024;
    const uint64_t xp = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)xp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(xp >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)(live * ksteps * 1024));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                             nb, 0x00020000);
  };
  const uint32_t xl = (uint32_t)opaque(lane) * 16u;
  auto load_a = [&](__amdgpu_buffer_rsrc_t xr, int ks) {
    const uint32_t off = ks < ksteps ? xl : 0x7fff0000u;
    return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, off, ks * 1024, 2));
  };
  f32x16 acc[kI2QT];
  const f32x16 acc0 = f32x16(kI8Magic);
  auto mfma = [&](int u, const f16x8& xv, const f16x8& bv, bool start) {
    typedef int i32x16 __attribute__((ext_vector_type(16)));
    const f32x16 cin = start ? acc0 : acc[u];
    acc[u] = __builtin_bit_cast(f32x16, __builtin_amdgcn_mfma_i32_32x32x32_i8(
        __builtin_bit_cast(i32x4, xv), __builtin_bit_cast(i32x4, bv),
        __builtin_bit_cast(i32x16, cin), 0, 0, 0));
  };
  // one k-step: its B fragments first (one LDS wait), then the MFMAs.  The
  // previous k-step's fragments stay allocated until this k-step's reads are
  // issued, so the new fragments never land in registers an MFMA issued just
  // ahead (and possibly still queued behind the partner wave's MFMAs) reads.
  // Defensive only: the measured hazard was the epilogue's (below); without
  // this (FX_I6_BPREV=0) 0 of 88 repetitions moved and the times were equal
  // (profiles/r04_img6_bprev_sweep.jsonl)
#ifndef FX_I6_BPREV
#define FX_I6_BPREV 1
#endif
  f16x8 bprev[kI2QT];
#pragma unroll
  for (int u = 0; u < kI2QT; ++u) bprev[u] = f16x8(0);
  auto kstep = [&](const f16x8& xv, int ks, bool start) {
    f16x8 bv[kI2QT];
#pragma unroll
    for (int u = 0; u < kI2QT; ++u) bv[u] = bfrag(ks, u);
    if constexpr (FX_I6_BPREV != 0) {
#pragma unroll
      for (int u = 0; u < kI2QT; ++u) asm volatile("" ::"v"(bprev[u]));
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kI2QT; ++u) mfma(u, xv, bv[u], start);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < kI2QT; ++u) bprev[u] = bv[u];
  };
  const int lr = wid * 32 + l32;  // the wave's row this lane notes (lanes 0-31)
  int64_t ti = blockIdx.x;
  __amdgpu_buffer_rsrc_t xr = x_rsrc(ti);
  f16x8 xa[XS];
#pragma unroll
  for (int s = 0; s < XS; ++s) xa[s] = load_a(xr, s);
  for (; ti < ntiles; ti += gridDim.x) {
    const int64_t r0 = tile_r0(ti);
    const int64_t tn = ti + gridDim.x;
    const __amdgpu_buffer_rsrc_t xn = x_rsrc(tn);
    // this tile's row terms, early (lanes 0-31: row r0 + wid * 32 + l32)
    const int64_t row = r0 + lr;
    const int64_t rowc = row < a.n ? row : a.n - 1;
    const f32x4 rsum = *reinterpret_cast<const f32x4*>(a.rowinfo + rowc * kI8RowInfo);
    const uint32_t crow = perm_row(a.perm_a, a.n, rowc);
    const uint32_t mword = a.mask != nullptr ? a.mask[crow >> 5] >> (crow & 31) : 1u;
    // k-step groups of XS: the first starts the accumulators, the last
    // refills from the next tile
    for (int g = 0; g < ngroups; ++g) {
      const bool last = g + 1 == ngroups;
#pragma unroll
      for (int s = 0; s < XS; ++s) {
        const int ks = g * XS + s;
        kstep(xa[s], ks, ks == 0);
        xa[s] = last ? load_a(xn, s) : load_a(xr, ks + XS);
      }
    }
    // the wave's 32 rows: terms, corpus rows and flags into its own LDS words
    if (lane < 4) sh->rflags[(lane >> 1) * 16 + wid * 2 + (lane & 1)] = 0u;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (h == 0) {
      const bool ok = row < a.n && (mword & 1u);
      const float y1 = METRIC == 1 ? rsum[1] : METRIC == 2 ? rsum[2] : rsum[3];
      i8_note_row(sh->rinfo, sh->rterm, sh->rext, sh->rflags, lr, rsum[0], y1, rsum[1], ok);
      sh->rrow[lr] = (uint32_t)a.row_base + crow;
    }
    // Every wave of the workgroup past its last MFMA before any epilogue
    // reads its accumulators.  Without this barrier the waves ran free and
    // the epilogue now and then read a product of the tile's last k-step
    // before the MFMA had written it: the same search repeated appended one
    // more or one fewer row for query lanes 16-31 of a tile (no padding of
    // s_nop after the MFMAs removed it, so the MFMA was still queued behind
    // the partner wave's on the SIMD's matrix pipe).  tools/race_check.py:
    // 0 of 88 repetitions move with it, 201 of 232 without; it costs
    // nothing on a single query (1.295 vs 1.300 ms for configs[1]).
#ifndef FX_I6_PRE_EPI  // experiment switch (tools/race_check.py builds):
#define FX_I6_PRE_EPI 1  // 0 no barrier, 1 barrier, 2 own loads drained, 3 64 wait states
#endif
    if constexpr (FX_I6_PRE_EPI == 1)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (FX_I6_PRE_EPI == 2)
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else if constexpr (FX_I6_PRE_EPI == 3)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" :::
                   "memory");
    else
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!(diag & 2))
      i8_epilogue<METRIC>(acc, sh->rinfo, sh->rterm, sh->rext, sh->rrow, sh->rflags, sh->qtab,
                          sh->qinf, a, q0, wid, h, l32, sh->seg, diag, segcap);
    xr = xn;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  filter_flush_segments<SEG, kI6Threads>(sh->seg, sh->segbase, a, q0, tid, segcap);
}

int launch_img6(const FilterArgs& a, int metric, hipStream_t stream) {
  if (a.num_tiles <= 0) return FX_OK;
  const size_t smem = img6_smem(a.dq);
  const void* fn = metric == FX_METRIC_COS  ? (const void*)filter_img6_kernel<2>
                   : metric == FX_METRIC_IP ? (const void*)filter_img6_kernel<1>
                                            : (const void*)filter_img6_kernel<0>;
  if (int rc = allow_lds(fn)) return rc;
  int cus = 0;
  if (int rc = device_cus(&cus)) return rc;
  const int64_t slices = (a.nq + fBQ - 1) / fBQ;
  // every slice's workgroups co-resident (one per CU): slices x G <= CUs
  int64_t bx = cus / (slices < cus ? slices : cus);
  if (bx < 1) bx = 1;
  if (bx > a.num_tiles) bx = a.num_tiles;
  for (int64_t y0 = 0; y0 < slices; y0 += 65535) {
    FilterArgs b = a;
    const int64_t yn = (slices - y0) < 65535 ? (slices - y0) : 65535;
    b.Qh = a.Qh + y0 * fBQ * 32;
    b.qinfo = a.qinfo + y0 * fBQ * kI8QInfo;
    b.thr = a.thr + y0 * fBQ;
    b.count = a.count + y0 * fBQ * kCountStride;
    b.cand = a.cand + y0 * fBQ * (int64_t)a.cap;
    if (a.cand_ub) b.cand_ub = a.cand_ub + y0 * fBQ * (int64_t)a.cap;
    b.nq = a.nq - y0 * fBQ;
    void* args[] = {(void*)&b};
    hipError_t e = hipLaunchKernel(fn, dim3((unsigned)bx, (unsigned)yn), dim3(kI6Threads), args,
                                   smem, stream);
    if (e != hipSuccess) {
      set_error("filter_img6_kernel launch: %s", hipGetErrorString(e));
      return FX_EHIP;
    }
  }
  return check_launch("filter_img6_kernel");
}
#endif  // FX_FILTER_BQ <= 128
#endif  // FX_FILTER_IMG3

#if FX_FILTER_IMG3
// [lb, ub] of a (row, query) pair from the fp16 product x, the row value rv
// (cosine max(|x|, 1e-12), IP |x|, L2 |x|^2; NaN: forced) and the query's
// {c1, c0, A, B} (filter_query_table)
template <int METRIC>
__device__ __forceinline__ void i4_bounds(float x, float rv, const f32x4& qc, float& lb,
                                          float& ub) {
  const float qc1 = qc[0], qc0 = qc[1], qA = qc[2], qB = qc[3];
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
    const float rt = 1.f / rv;
    const float dist = fmaf(x * rt, qc1, 0.5f);
    const float e = fmaf(qB, rt, qA);
    lb = dist - e;
    ub = dist + e;
  }
  if (!(qA <= 3.4e38f) || rv != rv) {  // forced: below / above every key
    lb = -__builtin_inff();
    ub = __builtin_nanf("");
  }
}

#endif

// ------------------------------ tiled image, both operands by LDS-DMA rings
#if !FX_FILTER_IMG3  // (the 256-query, 32-wide-K build only)
#undef FX_FILTER_IMG5
#define FX_FILTER_IMG5 0
#endif
#ifndef FX_FILTER_IMG5
#define FX_FILTER_IMG5 0
#endif
#if FX_FILTER_IMG5
//
// filter_img5_kernel: filter_img3_kernel with the image by LDS-DMA too and
// the appends straight to the candidate buffer:
//   * each wave DMAs its own 32-row tile's K chunk (2 KB) into a ring of
//     FX_I5_XA + 1 slots, FX_I5_XA chunks ahead, and reads its A fragments
//     back from where the DMA put them (lane L's 16 B at +16 L: no conflicts);
//     the image needs no barrier (a wave reads only its own pieces) and no
//     registers, so it runs deeper than register stages allow;
//   * a workgroup appends to its own region of each query's candidate
//     buffer, cap / gridDim.x slots from slot blockIdx.x * that, positions
//     from an LDS counter: no global atomic with a return value (which
//     would wait for the whole prefetched stream) and no flush.  A region
//     that fills marks its query overflowed (count bit 31): the exact
//     fallback recomputes it.  At the end every count is raised to cap, so
//     the rescoring walks every slot (empty ones are skipped).
#ifndef FX_I5_QA
#define FX_I5_QA 3
#endif
#ifndef FX_I5_XA
#define FX_I5_XA 4
#endif
#ifndef FX_I5_SCHED
#define FX_I5_SCHED 1  // fragment reads grouped ahead of each k-step's MFMAs
#endif
constexpr int kI5QSlots = FX_I5_QA + 1, kI5XSlots = FX_I5_XA + 1;
constexpr int kI5XBytes = fBM * fBK * 2;  // one image slot: every wave's 2 x 1 KB
static_assert(FX_I5_QA < FX_I5_XA, "img5: an image chunk is issued before its query chunk");
struct Img5Shared {
  unsigned char qring[kI5QSlots][kI3QBytes];
  unsigned char xring[kI5XSlots][kI5XBytes];
  float rinfo[fBM];
  float rterm[fBM];
  uint32_t rflags[2][kRowFlagWords];
  f32x4 qtab[fBQ];
  float2 qab[fBQ];
  uint32_t qcount[fBQ];  // this workgroup's appends per query
};
static_assert(sizeof(Img5Shared) <= 160 * 1024, "filter_img5_kernel: LDS over 160 KB");

template <int METRIC>
__device__ __forceinline__ void i5_epilogue(const f32x16 (&acc)[kI2QT], const float* rinfo,
                                            const float* rterm, const uint32_t* flags,
                                            const f32x4* qtab, const float2* qab,
                                            const FilterArgs& a, int64_t q0, int64_t r0, int wid,
                                            int h, int l32, uint32_t* qcount, uint32_t region,
                                            int diag) {
  const int lr0 = wid * 32 + 4 * h;
  f32x4 rv4[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) rv4[g] = *reinterpret_cast<const f32x4*>(rinfo + lr0 + 8 * g);
  const uint32_t fmask = flags[wid * 2 + h], smask = flags[16 + wid * 2 + h];
  uint32_t pm[kI2QT];
#pragma unroll
  for (int u = 0; u < kI2QT; ++u) {
    const float2 ab = qab[u * 32 + l32];
    const f32x2 na = {-ab.x, -ab.x}, nb = {-ab.y, -ab.y};
    uint32_t fail = 0u;
#pragma unroll
    for (int i = 7; i >= 0; --i) {
      const f32x4 r = rv4[i >> 1];
      const f32x2 rp = (i & 1) ? f32x2{r[2], r[3]} : f32x2{r[0], r[1]};
      const f32x2 xp = {acc[u][2 * i], acc[u][2 * i + 1]};
      const f32x2 dd = __builtin_elementwise_fma(na, rp, xp) + nb;
      fail = __builtin_amdgcn_alignbit(fail, __float_as_uint(dd[1]), 31);
      fail = __builtin_amdgcn_alignbit(fail, __float_as_uint(dd[0]), 31);
    }
    pm[u] = (diag & 1) ? 0u : (~fail | fmask) & ~smask & 0xffffu;
    if (q0 + u * 32 + l32 >= a.nq) pm[u] = 0u;
  }
  uint32_t any = 0u;
#pragma unroll
  for (int u = 0; u < kI2QT; ++u) any |= pm[u];
  if (__ballot(any != 0u) == 0ull) return;
  uint32_t pos[kI2QT];
#pragma unroll
  for (int u = 0; u < kI2QT; ++u)
    pos[u] = pm[u] != 0u ? atomicAdd(&qcount[u * 32 + l32], (uint32_t)__popc(pm[u])) : 0u;
  static_for<kI2QT>([&](auto uc) {
    constexpr int u = decltype(uc)::value;
    if (__ballot(pm[u] != 0u) == 0ull) return;
    const int qi = u * 32 + l32;
    // (opaque: per-query addresses hoisted out of the tile loop were spilled)
    const int64_t gq = q0 + (int)opaque((unsigned)qi);
    uint32_t bits = pm[u], p = pos[u];
    if (bits != 0u && p + (uint32_t)__popc(bits) > region)  // the region is full: overflowed
      atomicOr(&a.count[gq * kCountStride], 0x80000000u);
    const f32x4 qc = qtab[qi];
    uint64_t* cl = a.cand + (size_t)gq * a.cap + (size_t)blockIdx.x * region;
    uint64_t* cu = a.cand_ub != nullptr ? a.cand_ub + (size_t)gq * a.cap + (size_t)blockIdx.x * region
                                        : nullptr;
    while (bits != 0u && p < region) {
      const int j = __builtin_ctz(bits);
      bits &= bits - 1u;
      auto pick = [](float lo, float hi, uint32_t m) {
        return __uint_as_float((__float_as_uint(hi) & m) | (__float_as_uint(lo) & ~m));
      };
      const uint32_t m0 = 0u - ((uint32_t)j & 1u), m1 = 0u - (((uint32_t)j >> 1) & 1u);
      const uint32_t m2 = 0u - (((uint32_t)j >> 2) & 1u), m3 = 0u - (((uint32_t)j >> 3) & 1u);
      float v8[8], v4[4], v2[2];
#pragma unroll
      for (int i = 0; i < 8; ++i) v8[i] = pick(acc[u][2 * i], acc[u][2 * i + 1], m0);
#pragma unroll
      for (int i = 0; i < 4; ++i) v4[i] = pick(v8[2 * i], v8[2 * i + 1], m1);
#pragma unroll
      for (int i = 0; i < 2; ++i) v2[i] = pick(v4[2 * i], v4[2 * i + 1], m2);
      const float x = pick(v2[0], v2[1], m3);
      const int lr = lr0 + (j & 3) + 8 * (j >> 2);
      const float rv = rinfo[lr];
      float lb, ub;
      if constexpr (METRIC == 2) {  // (i4_bounds recomputes 1 / rv; the row's is in LDS)
        const float rt = rterm[lr];
        const float dist = fmaf(x * rt, qc[0], 0.5f);
        const float e = fmaf(qc[3], rt, qc[2]);
        lb = dist - e;
        ub = dist + e;
        if (!(qc[2] <= 3.4e38f) || rv != rv) {
          lb = -__builtin_inff();
          ub = __builtin_nanf("");
        }
      } else {
        i4_bounds<METRIC>(x, rv, qc, lb, ub);
      }
      const uint32_t grow = (uint32_t)(a.row_base + r0) + (uint32_t)lr;
      if (cu != nullptr) {
        cl[p] = make_comp(lb, grow);
        cu[p] = make_comp(ub, grow);
      } else {
        cl[p] = make_comp(ub, grow);
      }
      ++p;
    }
  });
}

template <int N>
__device__ __forceinline__ void i5_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

template <int METRIC>
__global__ void __launch_bounds__(fThreads, fWaves / 4) filter_img5_kernel(FilterArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  Img5Shared* sh = reinterpret_cast<Img5Shared*>(smem);
#ifdef FX_DIAG_BUILD  // FX_FILTER_DIAG as filter_img3_kernel
  const int diag = a.diag;
#else
  constexpr int diag = 0;
#endif
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, l32 = lane & 31;
  const int64_t q0 = (int64_t)blockIdx.y * fBQ;
  const int nch = (a.d + fBK - 1) / fBK;
  const int ksteps = (a.d + 15) / 16;
  const int64_t ntile32 = (a.n + 31) / 32;
  const uint32_t region = (uint32_t)a.cap / gridDim.x;
  if ((int64_t)blockIdx.x >= a.num_tiles) return;
  filter_query_table<METRIC>(a, q0, sh->qtab, sh->qab, tid, fThreads);
  for (int q = tid; q < fBQ; q += fThreads) sh->qcount[q] = 0u;

  const __amdgpu_buffer_rsrc_t qr = [&] {
    const uint64_t qp = reinterpret_cast<uint64_t>(a.Qh + q0 * 32);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)qp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(qp >> 32));
    const int nb = __builtin_amdgcn_readfirstlane(
        (int)(((int64_t)(a.dq / 32 - 1) * a.qstride + fBQ) * 64));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                             nb, 0x00020000);
  }();
  uint32_t qv[kI3QDma];
#pragma unroll
  for (int i = 0; i < kI3QDma; ++i) {
    const int j = wid * kI3QDma + i;
    const int q = 16 * j + (lane >> 2);
    qv[i] = (uint32_t)(q * 64 + (((lane & 3) ^ ((q >> 2) & 3)) * 16));
  }
  auto issue_q = [&](int c, int slot) {
    if (diag & 8) return;
    unsigned char* st = sh->qring[slot];
#pragma unroll
    for (int i = 0; i < kI3QDma; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(qr, (i3_lds_ptr)(st + (wid * kI3QDma + i) * 1024), 16,
                                               qv[i], (int)(c * a.qstride * 64), 0, 0);
  };
  auto x_rsrc = [&](int64_t ti) {
    const int64_t t32 = (a.tile_start + ti * a.tile_stride) * (fBM / 32) + wid;
    const int64_t live = (ti < a.num_tiles && t32 < ntile32) ? 1 : 0;
    const unsigned char* base = reinterpret_cast<const unsigned char*>(a.X) +
                                (live ? t32 : 0) * (int64_t)ksteps * 1024;
    const uint64_t xp = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)xp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(xp >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)(live * ksteps * 1024));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                             nb, 0x00020000);
  };
  const uint32_t xl = (uint32_t)opaque(lane) * 16u;
  // this wave's K chunk c of its 32-row tile into image slot `slot`: k-step
  // s lands at +(2 w + s) KB, lane L's 16 B at +16 L (its A fragment)
  auto issue_x = [&](__amdgpu_buffer_rsrc_t xr, int c, int slot) {
    unsigned char* st = sh->xring[slot] + wid * 2048;
#pragma unroll
    for (int s = 0; s < kI2KS; ++s) {
      const int ks = c * kI2KS + s;
      const uint32_t off = (ks < ksteps && !(diag & 32)) ? xl : 0x7fff0000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (i3_lds_ptr)(st + s * 1024), 16, off, ks * 1024,
                                               0, 2 /* nt */);
    }
  };
  uint32_t bq[kI2KS];
#pragma unroll
  for (int s = 0; s < kI2KS; ++s) {
    const int Q = (int)opaque((unsigned)l32);
    bq[s] = (uint32_t)(Q * 64 + (((2 * s + h) ^ ((Q >> 2) & 3)) * 16));
  }
  const uint32_t xrd = (uint32_t)wid * 2048u + xl;  // this lane's A fragment in an image slot
  f32x16 acc[kI2QT];
  auto compute = [&](int qs, int xs) {
    if (diag & 4) return;
    const unsigned char* st = sh->qring[qs];
    const unsigned char* sx = sh->xring[xs];
#pragma unroll
    for (int s = 0; s < kI2KS; ++s) {
      const f16x8 av = *reinterpret_cast<const f16x8*>(sx + xrd + s * 1024);
      f16x8 bv[kI2QT];
#pragma unroll
      for (int u = 0; u < kI2QT; ++u)
        bv[u] = *reinterpret_cast<const f16x8*>(st + bq[s] + u * 32 * 64);
#pragma unroll
      for (int u = 0; u < kI2QT; ++u)
        acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bv[u], acc[u], 0, 0, 0);
#if FX_I5_SCHED
      // the k-step's 9 fragment reads first, then its 8 MFMAs: the reads'
      // latency is paid once per k-step, not before every MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 9, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
#endif
    }
  };

  // ---- prologue: query chunks 0 .. QA-1 and image chunks 0 .. XA-1
  int qc = 0, qslot = 0;
#pragma unroll
  for (int i = 0; i < FX_I5_QA; ++i) {
    issue_q(qc, qslot);
    qc = qc + 1 == nch ? 0 : qc + 1;
    qslot = qslot + 1 == kI5QSlots ? 0 : qslot + 1;
  }
  int64_t xt = blockIdx.x;
  int xc = 0, xslot = 0;
  __amdgpu_buffer_rsrc_t xr = x_rsrc(xt);
#pragma unroll
  for (int i = 0; i < FX_I5_XA; ++i) {
    issue_x(xr, xc, xslot);
    xslot = xslot + 1 == kI5XSlots ? 0 : xslot + 1;
    if (++xc == nch) {
      xc = 0;
      xt += gridDim.x;
      xr = x_rsrc(xt);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (once: the prologue's order differs)
  int rq = 0, rx = 0;  // slots the next step reads
  int par = 0;
  for (int64_t ti = blockIdx.x; ti < a.num_tiles; ti += gridDim.x, par ^= 1) {
    const int64_t r0 = (a.tile_start + ti * a.tile_stride) * fBM;
    if (tid < kRowFlagWords) sh->rflags[par][tid] = 0u;
#pragma unroll
    for (int u = 0; u < kI2QT; ++u) acc[u] = f32x16(0.f);
    float rsum = 0.f;
    uint32_t mword = 0u;
    for (int c = 0; c < nch; ++c) {
      // query chunk c landed for every wave (this wave's image chunk c, issued
      // a step before it, with it), and every wave done with the slots refilled
      if (diag & 16)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else
        i5_wait_barrier<kI2KS + (FX_I5_QA - 1) * (kI3QDma + kI2KS)>();
      issue_q(qc, qslot);
      qc = qc + 1 == nch ? 0 : qc + 1;
      qslot = qslot + 1 == kI5QSlots ? 0 : qslot + 1;
      issue_x(xr, xc, xslot);
      xslot = xslot + 1 == kI5XSlots ? 0 : xslot + 1;
      if (++xc == nch) {
        xc = 0;
        xt += gridDim.x;
        xr = x_rsrc(xt);
      }
      if (c == 0) {  // the rows' image sums and mask words of this tile
        const int lr = tid & (fBM - 1);
        const int64_t row = r0 + lr < a.n ? r0 + lr : a.n - 1;
        rsum = a.rowinfo[row];
        const bool masked = a.mask != nullptr;
        const uint32_t* mp = masked ? a.mask + (row >> 5)
                                    : reinterpret_cast<const uint32_t*>(a.rowinfo) + row;
        mword = *mp | (masked ? 0u : ~0u);
      }
      compute(rq, rx);
      rq = rq + 1 == kI5QSlots ? 0 : rq + 1;
      rx = rx + 1 == kI5XSlots ? 0 : rx + 1;
    }
    if (tid < fBM) {  // one thread per row: bound factor, flags
      const int lr = (int)opaque((unsigned)tid);
      const int64_t row = r0 + lr;
      bool ok = row < a.n && ((mword >> (row & 31)) & 1u);
      const float s = ok ? rsum : 0.f;
      float rv;
      if constexpr (METRIC == 0) {
        rv = s;
      } else if constexpr (METRIC == 1) {
        rv = sqrtf(s);
      } else {
        rv = fmaxf(sqrtf(s), 1e-12f);
      }
      if (!(s <= 3.4e38f)) rv = __builtin_nanf("");
      filter_note_row<METRIC, 1>(sh->rinfo, sh->rterm, sh->rflags[par], lr, rv, ok);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (diag & 2) {
      if (acc[0][0] == 1.2345f) a.count[0] = 7;
    } else {
      i5_epilogue<METRIC>(acc, sh->rinfo, sh->rterm, sh->rflags[par], sh->qtab, sh->qab, a, q0,
                          r0, wid, h, l32, sh->qcount, region, diag);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // every count at least cap: the rescoring walks every slot of the regions
  for (int q = tid; q < fBQ; q += fThreads)
    if (q0 + q < a.nq) atomicMax(&a.count[(q0 + q) * kCountStride], (uint32_t)a.cap);
}

static int launch_img5(const FilterArgs& a, int metric, hipStream_t stream) {
  const size_t smem = sizeof(Img5Shared);
  const void* fn = metric == FX_METRIC_COS ? (const void*)filter_img5_kernel<2>
                   : metric == FX_METRIC_IP ? (const void*)filter_img5_kernel<1>
                                            : (const void*)filter_img5_kernel<0>;
  if (int rc = allow_lds(fn)) return rc;
  int cus = 0;
  int rc = device_cus(&cus);
  if (rc) return rc;
  const int64_t qtiles = (a.nq + fBQ - 1) / fBQ;
  int64_t bx = cus;
  if (bx > a.num_tiles) bx = a.num_tiles;
  for (int64_t y0 = 0; y0 < qtiles; y0 += 65535) {
    FilterArgs b = a;
    const int64_t yn = (qtiles - y0) < 65535 ? (qtiles - y0) : 65535;
    b.Qh = a.Qh + y0 * fBQ * 32;
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
      set_error("filter_img5_kernel launch: %s", hipGetErrorString(e));
      return FX_EHIP;
    }
  }
  return check_launch("filter_img5_kernel");
}
#endif  // FX_FILTER_IMG5

// ------------------------- tiled image, one wave per SIMD, 64-row wave tiles
#if !FX_FILTER_IMG3  // (the 256-query, 32-wide-K build only)
#undef FX_FILTER_IMG4
#define FX_FILTER_IMG4 0
#endif
#ifndef FX_FILTER_IMG4
#define FX_FILTER_IMG4 0
#endif
#if FX_FILTER_IMG4
//
// filter_img4_kernel: filter_img3_kernel with 4 waves of 512 registers (one
// per SIMD) instead of 8 of 256.  Wave w owns rows 64 w .. + 63 of the
// 256-row tile (two 32-row MFMA row tiles) against all 256 queries: 256
// accumulator registers, and every B fragment read from the query ring feeds
// two MFMAs (half the LDS reads per MFMA).  The register room holds
// FX_I4_XS image chunks in flight.  Appends store the raw product, the row
// value and the row in the LDS segment; their bounds are computed when the
// segments are flushed.
#ifndef FX_I4_XS
#define FX_I4_XS 3
#endif
#ifndef FX_I4_SEG
#define FX_I4_SEG 20  // LDS append entries per query (overflow: global slots)
#endif
constexpr int kI4Waves = 4, kI4Threads = 64 * kI4Waves;
struct Img4Shared {
  unsigned char qring[kI3Slots][kI3QBytes];
  float rinfo[fBM];
  uint32_t rflags[2][kRowFlagWords];
  f32x4 qtab[fBQ];
  float2 qab[fBQ];
  float stage[kI4Waves][16 * 64];  // per wave: one query tile's accumulators, [element][lane]
  uint32_t seg[fBQ + 3 * fBQ * FX_I4_SEG];  // counters, then raw entries {x, rv, row}
  uint32_t segbase[fBQ];
  float rterm[fBM];  // (cosine: written by filter_note_row, the bounds use 1 / rv)
};
static_assert(sizeof(Img4Shared) <= 160 * 1024, "filter_img4_kernel: LDS over 160 KB");
constexpr int kI4QDma = kI3QBytes / 1024 / kI4Waves;  // 1-KB query DMAs per wave per chunk
constexpr int kI4XLd = 2 * kI2KS;                     // image loads per wave per chunk
static_assert(kI4QDma * 1024 * kI4Waves == kI3QBytes && kI4Waves * 64 == fBM, "img4 tiling");

// One accumulator element, read from its AGPR by v_accvgpr_read: a plain
// VALU use makes the allocator copy whole accumulator tuples into VGPRs
// (and spill them); the "a" operand keeps them where the MFMAs wrote them.
// (The epilogue runs behind the tile's last barrier, far past the MFMA's
// write latency.)
__device__ __forceinline__ float acc_rd(float v) {
  float r;
  asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(v));
  return r;
}

// Pass test and appends of the 32-row group g of the tile (lanes' rows
// 32 g + 4 h + (j & 3) + 8 (j >> 2)) against all kI2QT query tiles.  A query
// tile with a pass has its accumulators staged in the wave's LDS rows
// (stage[element][lane]); each lane then walks its set bits with dynamic
// LDS reads (a dynamic register index would be scratch).
template <int METRIC>
__device__ __forceinline__ void i4_epilogue(const f32x16 (&acc)[kI2QT], int g, const float* rinfo,
                                            const uint32_t* flags, const f32x4* qtab,
                                            const float2* qab, const FilterArgs& a, int64_t q0,
                                            int64_t r0, int lane, float* stage, uint32_t* seg,
                                            int diag) {
  constexpr int SEG = FX_I4_SEG;
  const int h = lane >> 5, l32 = lane & 31;
  const int lr0 = g * 32 + 4 * h;
  f32x4 rv4[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) rv4[i] = *reinterpret_cast<const f32x4*>(rinfo + lr0 + 8 * i);
  const uint32_t fmask = flags[g * 2 + h], smask = flags[16 + g * 2 + h];
  uint32_t pm[kI2QT];
#pragma unroll
  for (int u = 0; u < kI2QT; ++u) {
    const float2 ab = qab[u * 32 + l32];
    const f32x2 na = {-ab.x, -ab.x}, nb = {-ab.y, -ab.y};
    uint32_t fail = 0u;
#pragma unroll
    for (int i = 7; i >= 0; --i) {
      const f32x4 r = rv4[i >> 1];
      const f32x2 rp = (i & 1) ? f32x2{r[2], r[3]} : f32x2{r[0], r[1]};
      const f32x2 xp = {acc_rd(acc[u][2 * i]), acc_rd(acc[u][2 * i + 1])};
      const f32x2 dd = __builtin_elementwise_fma(na, rp, xp) + nb;
      fail = __builtin_amdgcn_alignbit(fail, __float_as_uint(dd[1]), 31);
      fail = __builtin_amdgcn_alignbit(fail, __float_as_uint(dd[0]), 31);
    }
    pm[u] = (diag & 1) ? 0u : (~fail | fmask) & ~smask & 0xffffu;
    if (q0 + u * 32 + l32 >= a.nq) pm[u] = 0u;
  }
  uint32_t any = 0u;
#pragma unroll
  for (int u = 0; u < kI2QT; ++u) any |= pm[u];
  if (__ballot(any != 0u) == 0ull) return;
  // every query tile's segment slots at once (LDS atomics in flight together)
  uint32_t pos[kI2QT];
#pragma unroll
  for (int u = 0; u < kI2QT; ++u)
    pos[u] = pm[u] != 0u ? atomicAdd(&seg[u * 32 + l32], (uint32_t)__popc(pm[u])) : 0u;
  const uint32_t grow0 = (uint32_t)(a.row_base + r0);
  static_for<kI2QT>([&](auto uc) {
    constexpr int u = decltype(uc)::value;
    if (__ballot(pm[u] != 0u) == 0ull) return;
#pragma unroll
    for (int j = 0; j < 16; ++j) stage[j * 64 + lane] = acc_rd(acc[u][j]);
    const int qi = u * 32 + l32;
    uint32_t bits = pm[u], p = pos[u], gp = ~0u;
    while (bits != 0u) {
      const int j = __builtin_ctz(bits);
      const uint32_t rest = bits;
      bits &= bits - 1u;
      const float x = stage[j * 64 + lane];
      const int lr = lr0 + (j & 3) + 8 * (j >> 2);
      const float rv = rinfo[lr];
      const uint32_t grow = grow0 + (uint32_t)lr;
      if (p < (uint32_t)SEG) {  // raw: the bounds are computed at the flush
        uint32_t* e = seg + fBQ + 3 * (qi * SEG + p);
        e[0] = __float_as_uint(x);
        e[1] = __float_as_uint(rv);
        e[2] = grow;
      } else {  // rare: past the segment, global slots for the lane's remaining passes
        const int64_t gq = q0 + qi;
        if (gp == ~0u) gp = atomicAdd(&a.count[gq * kCountStride], (uint32_t)__popc(rest));
        if (gp < (uint32_t)a.cap) {
          float lb, ub;
          i4_bounds<METRIC>(x, rv, qtab[qi], lb, ub);
          const size_t slot = (size_t)gq * a.cap + gp;
          if (a.cand_ub != nullptr) {
            a.cand[slot] = make_comp(lb, grow);
            a.cand_ub[slot] = make_comp(ub, grow);
          } else {
            a.cand[slot] = make_comp(ub, grow);
          }
        }
        ++gp;
      }
      ++p;
    }
  });
}

// i4_epilogue's segments to the candidate buffer: one global atomic per
// query reserves the slots; each raw entry {x, rv, row} becomes its bounds.
template <int METRIC>
__device__ __forceinline__ void i4_flush(uint32_t* seg, uint32_t* base, const f32x4* qtab,
                                         const FilterArgs& a, int64_t q0, int tid) {
  constexpr int SEG = FX_I4_SEG;
  __syncthreads();
  for (int q = tid; q < fBQ; q += kI4Threads) {
    const uint32_t n = seg[q] < (uint32_t)SEG ? seg[q] : (uint32_t)SEG;
    seg[q] = n;
    base[q] = n != 0u && q0 + q < a.nq ? atomicAdd(&a.count[(q0 + q) * kCountStride], n) : 0u;
  }
  __syncthreads();
  for (int i = tid; i < fBQ * SEG; i += kI4Threads) {
    const int q = i / SEG, j = i % SEG;
    if ((uint32_t)j >= seg[q]) continue;
    const uint32_t p = base[q] + (uint32_t)j;
    if (p >= (uint32_t)a.cap) continue;
    const uint32_t* e = seg + fBQ + 3 * i;
    float lb, ub;
    i4_bounds<METRIC>(__uint_as_float(e[0]), __uint_as_float(e[1]), qtab[q], lb, ub);
    const size_t slot = (size_t)(q0 + q) * a.cap + p;
    if (a.cand_ub != nullptr) {
      a.cand[slot] = make_comp(lb, e[2]);
      a.cand_ub[slot] = make_comp(ub, e[2]);
    } else {
      a.cand[slot] = make_comp(ub, e[2]);
    }
  }
}

template <int METRIC>
__global__ void __launch_bounds__(kI4Threads, 1) filter_img4_kernel(FilterArgs a) {
  constexpr int XS = FX_I4_XS;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  Img4Shared* sh = reinterpret_cast<Img4Shared*>(smem);
#ifdef FX_DIAG_BUILD  // FX_FILTER_DIAG as filter_img3_kernel
  const int diag = a.diag;
#else
  constexpr int diag = 0;
#endif
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, l32 = lane & 31;
  const int64_t q0 = (int64_t)blockIdx.y * fBQ;
  const int nch = ((a.d + fBK - 1) / fBK + XS - 1) / XS * XS;
  const int ksteps = (a.d + 15) / 16;
  const int64_t ntile32 = (a.n + 31) / 32;
  if ((int64_t)blockIdx.x >= a.num_tiles) return;
  filter_query_table<METRIC>(a, q0, sh->qtab, sh->qab, tid, kI4Threads);
  for (int q = tid; q < fBQ; q += kI4Threads) sh->seg[q] = 0u;
  // the ring starts zeroed: a slot a chunk past the query tile's padding
  // never receives (its DMA is dropped) then holds finite values
  for (int i = tid; i < kI3Slots * kI3QBytes / 16; i += kI4Threads)
    reinterpret_cast<i32x4*>(sh->qring)[i] = i32x4(0);
  __syncthreads();

  const __amdgpu_buffer_rsrc_t qr = [&] {
    const uint64_t qp = reinterpret_cast<uint64_t>(a.Qh + q0 * 32);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)qp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(qp >> 32));
    const int nb = __builtin_amdgcn_readfirstlane(
        (int)(((int64_t)(a.dq / 32 - 1) * a.qstride + fBQ) * 64));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                             nb, 0x00020000);
  }();
  const int qchunks = a.dq / 32;  // chunks the query tile holds
  uint32_t qv[kI4QDma];
#pragma unroll
  for (int i = 0; i < kI4QDma; ++i) {
    const int j = wid * kI4QDma + i;
    const int q = 16 * j + (lane >> 2);
    qv[i] = (uint32_t)(q * 64 + (((lane & 3) ^ ((q >> 2) & 3)) * 16));
  }
  auto issue_q = [&](int c, int slot) {
    if (diag & 8) return;
    unsigned char* st = sh->qring[slot];
#pragma unroll
    for (int i = 0; i < kI4QDma; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          qr, (i3_lds_ptr)(st + (wid * kI4QDma + i) * 1024), 16,
          c < qchunks ? qv[i] : 0x7fff0000u, (int)(c * a.qstride * 64), 0, 0);
  };
  // this wave's two 32-row tiles (adjacent in the image: one descriptor)
  auto x_rsrc = [&](int64_t ti) {
    const int64_t t32 = (a.tile_start + ti * a.tile_stride) * (fBM / 32) + 2 * wid;
    int64_t live = ti < a.num_tiles ? ntile32 - t32 : 0;
    live = live < 0 ? 0 : live > 2 ? 2 : live;
    const unsigned char* base = reinterpret_cast<const unsigned char*>(a.X) +
                                (live ? t32 : 0) * (int64_t)ksteps * 1024;
    const uint64_t xp = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)xp);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(xp >> 32));
    const int nb = __builtin_amdgcn_readfirstlane((int)(live * ksteps * 1024));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                             nb, 0x00020000);
  };
  const uint32_t xl = (uint32_t)opaque(lane) * 16u;
  typedef f16x8 XA[2][kI2KS];
  auto load_x = [&](XA& xa, __amdgpu_buffer_rsrc_t xr, int c) {
    if (diag & 32) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < kI2KS; ++s) xa[t][s] = f16x8((_Float16)0.f);
      return;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int s = 0; s < kI2KS; ++s) {
        const int ks = c * kI2KS + s;  // wave-uniform: past the row end reads zeros
        const uint32_t off = ks < ksteps ? xl + (uint32_t)(t * ksteps * 1024) : 0x7fff0000u;
        xa[t][s] = __builtin_bit_cast(
            f16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, off, ks * 1024, 2 /* nt */));
      }
    }
  };
  uint32_t bq[kI2KS];
#pragma unroll
  for (int s = 0; s < kI2KS; ++s) {
    const int Q = (int)opaque((unsigned)l32);
    bq[s] = (uint32_t)(Q * 64 + (((2 * s + h) ^ ((Q >> 2) & 3)) * 16));
  }
  f32x16 acc[2][kI2QT];
  auto compute = [&](const XA& xa, int slot) {
    if (diag & 4) {
      if (xa[0][0][0] == (_Float16)1.2345f && xa[1][kI2KS - 1][7] == (_Float16)2.f) a.count[0] = 7;
      return;
    }
    const unsigned char* st = sh->qring[slot];
#pragma unroll
    for (int s = 0; s < kI2KS; ++s) {
      f16x8 bv[kI2QT];
#pragma unroll
      for (int u = 0; u < kI2QT; ++u)
        bv[u] = *reinterpret_cast<const f16x8*>(st + bq[s] + u * 32 * 64);
#pragma unroll
      for (int u = 0; u < kI2QT; ++u) {
        acc[0][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa[0][s], bv[u], acc[0][u], 0, 0, 0);
        acc[1][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa[1][s], bv[u], acc[1][u], 0, 0, 0);
      }
    }
  };

  int qc = 0, qslot = 0;
#pragma unroll
  for (int i = 0; i < FX_I3_QA; ++i) {
    issue_q(qc, qslot);
    qc = qc + 1 == nch ? 0 : qc + 1;
    qslot = qslot + 1 == kI3Slots ? 0 : qslot + 1;
  }
  XA xa[XS];
  int64_t xt = blockIdx.x;
  int xc = 0;
  __amdgpu_buffer_rsrc_t xr = x_rsrc(xt);
  static_for<XS>([&](auto sc) {
    load_x(xa[decltype(sc)::value], xr, xc);
    if (++xc == nch) {
      xc = 0;
      xt += gridDim.x;
      xr = x_rsrc(xt);
    }
  });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int rslot = 0;
  int par = 0;
  for (int64_t ti = blockIdx.x; ti < a.num_tiles; ti += gridDim.x, par ^= 1) {
    const int64_t r0 = (a.tile_start + ti * a.tile_stride) * fBM;
    if (tid < kRowFlagWords) sh->rflags[par][tid] = 0u;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < kI2QT; ++u) acc[t][u] = f32x16(0.f);
    float rsum = 0.f;
    uint32_t mword = 0u;
    auto step = [&](int c, auto sc) {
      constexpr int S = decltype(sc)::value;
      if (diag & 16)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else
        i3_wait_barrier<kI4XLd + (FX_I3_QA - 1) * (kI4QDma + kI4XLd)>();
      issue_q(qc, qslot);
      qc = qc + 1 == nch ? 0 : qc + 1;
      qslot = qslot + 1 == kI3Slots ? 0 : qslot + 1;
      if (S == 0 && c == 0) {  // the rows' image sums and mask words of this tile
        const int64_t row = r0 + tid < a.n ? r0 + tid : a.n - 1;
        rsum = a.rowinfo[row];
        const bool masked = a.mask != nullptr;
        const uint32_t* mp = masked ? a.mask + (row >> 5)
                                    : reinterpret_cast<const uint32_t*>(a.rowinfo) + row;
        mword = *mp | (masked ? 0u : ~0u);
      }
      compute(xa[S], rslot);
      rslot = rslot + 1 == kI3Slots ? 0 : rslot + 1;
      load_x(xa[S], xr, xc);
      if (++xc == nch) {
        xc = 0;
        xt += gridDim.x;
        xr = x_rsrc(xt);
      }
    };
    for (int c = 0; c < nch; c += XS) static_for<XS>([&](auto sc) { step(c, sc); });
    {  // one thread per row: bound factor, flags
      const int lr = (int)opaque((unsigned)tid);
      const int64_t row = r0 + lr;
      bool ok = row < a.n && ((mword >> (row & 31)) & 1u);
      const float s = ok ? rsum : 0.f;
      float rv;
      if constexpr (METRIC == 0) {
        rv = s;
      } else if constexpr (METRIC == 1) {
        rv = sqrtf(s);
      } else {
        rv = fmaxf(sqrtf(s), 1e-12f);
      }
      if (!(s <= 3.4e38f)) rv = __builtin_nanf("");
      filter_note_row<METRIC, 1>(sh->rinfo, sh->rterm, sh->rflags[par], lr, rv, ok);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (diag & 2) {
      if (acc[0][0][0] == 1.2345f) a.count[0] = 7;
    } else {
      const int ol = (int)opaque((unsigned)lane);
      i4_epilogue<METRIC>(acc[0], 2 * wid, sh->rinfo, sh->rflags[par], sh->qtab, sh->qab, a, q0,
                          r0, ol, sh->stage[wid], sh->seg, diag);
      i4_epilogue<METRIC>(acc[1], 2 * wid + 1, sh->rinfo, sh->rflags[par], sh->qtab, sh->qab, a,
                          q0, r0, ol, sh->stage[wid], sh->seg, diag);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  i4_flush<METRIC>(sh->seg, sh->segbase, sh->qtab, a, q0, tid);
}

static int launch_img4(const FilterArgs& a, int metric, hipStream_t stream) {
  const size_t smem = sizeof(Img4Shared);
  const void* fn = metric == FX_METRIC_COS ? (const void*)filter_img4_kernel<2>
                   : metric == FX_METRIC_IP ? (const void*)filter_img4_kernel<1>
                                            : (const void*)filter_img4_kernel<0>;
  if (int rc = allow_lds(fn)) return rc;
  int cus = 0;
  int rc = device_cus(&cus);
  if (rc) return rc;
  const int64_t qtiles = (a.nq + fBQ - 1) / fBQ;
  int64_t bx = cus;
  if (bx > a.num_tiles) bx = a.num_tiles;
  for (int64_t y0 = 0; y0 < qtiles; y0 += 65535) {
    FilterArgs b = a;
    const int64_t yn = (qtiles - y0) < 65535 ? (qtiles - y0) : 65535;
    b.Qh = a.Qh + y0 * fBQ * 32;
    b.qinfo = a.qinfo + y0 * fBQ * 4;
    b.thr = a.thr + y0 * fBQ;
    b.count = a.count + y0 * fBQ * kCountStride;
    b.cand = a.cand + y0 * fBQ * (int64_t)a.cap;
    if (a.cand_ub) b.cand_ub = a.cand_ub + y0 * fBQ * (int64_t)a.cap;
    b.nq = a.nq - y0 * fBQ;
    void* args[] = {(void*)&b};
    hipError_t e = hipLaunchKernel(fn, dim3((unsigned)bx, (unsigned)yn), dim3(kI4Threads), args,
                                   smem, stream);
    if (e != hipSuccess) {
      set_error("filter_img4_kernel launch: %s", hipGetErrorString(e));
      return FX_EHIP;
    }
  }
  return check_launch("filter_img4_kernel");
}
#endif  // FX_FILTER_IMG4

#ifndef FX_FILTER_SPLIT  // measured slower (6.48 vs 6.35 ms for configs[2], same box)
#define FX_FILTER_SPLIT 0
#endif

template <typename XT, int METRIC, bool IMG>
__global__ void __launch_bounds__(fThreads, fWaves * FX_FILTER_BPC / 4) filter_kernel(FilterArgs a) {
  static_assert(!IMG || sizeof(XT) == 2, "the filter image is fp16");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  FilterShared* sh = reinterpret_cast<FilterShared*>(smem);
  const int tid = threadIdx.x;
  filter_query_table<METRIC>(a, (int64_t)blockIdx.y * fBQ, sh->qtab, sh->qab, tid, fThreads);
  // (the first tile's barriers order these writes before the epilogue reads)
#ifdef FX_DIAG_BUILD
  const int diag = a.diag;
#else
  constexpr int diag = 0;
#endif
  // wave-uniform role: the whole tile loop is instantiated per role, so the
  // loop holds no join (both copies run the same count of barriers)
  if (FX_FILTER_SPLIT && __builtin_amdgcn_readfirstlane(tid >> 6) >= fWaves / 2)
    filter_tiles<XT, METRIC, IMG, true>(a, smem, tid, diag);
  else
    filter_tiles<XT, METRIC, IMG, false>(a, smem, tid, diag);
}

#ifdef FX_DIAG_BUILD  // rejected variant, tools/ builds only
// ------------------------------------------------------------- LDS-DMA ring
//
// The same filter with every operand staged by LDS-DMA (buffer_load ... lds):
// no prefetch registers, a 3-deep ring of K-chunk stages (X rows and the query
// tile, 48 KB per stage for f32 rows), one raw s_barrier per chunk behind a
// COUNTED vmcnt so two stages stay in flight across it (a __syncthreads()
// would drain them: cdna_hip_programming.md §5 "Pipelining across barriers").
// The stage sequence runs on across tiles, so the next tile's first chunks
// stream in while a tile's epilogue runs.  Rows are converted to fp16 at
// fragment-read time (f32 corpora) or read as they are (f16 corpora: exact).
// LDS images are XOR-swizzled by 16-B piece (the DMA writes lane L at
// base + 16 L; the swizzle is applied to the global address) so fragment
// reads are bank-conflict free.
namespace ring {
#ifndef FX_RING_WAVES
#define FX_RING_WAVES (FX_FILTER_BQ >= 256 ? 16 : 8)  // 64 or 32 accumulator registers per wave
#endif
constexpr int kBM = 256, kBQ = FX_FILTER_BQ, kBK = 32, kStages = 3, kWaves = FX_RING_WAVES;
constexpr int kThreads = kWaves * 64;
constexpr int kRG = 4;                  // 64-row groups
constexpr int kQG = kWaves / kRG;       // query groups
constexpr int kQT = kBQ / kQG / 32;     // 32-query tiles per wave
template <typename XT>
struct Lay {
  static constexpr int xrow = kBK * (int)sizeof(XT);  // bytes per row per stage
  static constexpr int xbytes = kBM * xrow;
  static constexpr int qbytes = kBQ * kBK * 2;
  static constexpr int stage = xbytes + qbytes;
  // 1 KB DMA instructions per wave and stage; every wave issues the same
  // number (the counted waits rely on it), surplus ones land in a dummy KB
  static constexpr int xblocks = xbytes / 1024, qblocks = qbytes / 1024;
  static constexpr int xdma = (xblocks + kWaves - 1) / kWaves;
  static constexpr int qdma = (qblocks + kWaves - 1) / kWaves;
  static constexpr int ndma = xdma + qdma;
  static constexpr int rinfo = kStages * stage;
  static constexpr int rterm = rinfo + kBM * 4;
  static constexpr int rflags = rterm + kBM * 4;  // [2][kRowFlagWords] by tile parity
  static constexpr int qtab = rflags + 2 * kRowFlagWords * 4;
  static constexpr int qab = qtab + kBQ * 16;
  static constexpr int dummy = qab + kBQ * 8;
  static constexpr int total = dummy + 1024;
};

typedef __attribute__((address_space(3))) void* lds_ptr;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, int64_t bytes) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0,
                                           nb, 0x00020000);
}

// Issue the DMA of K chunk c of the tile at row r0 (and of the query tile)
// into stage buffer sb.  Rows past n read as zeros (descriptor size), pieces
// past d through an offset beyond it; a tile index past the end gets an empty
// descriptor, so every wave always issues exactly Lay::ndma instructions.
template <typename XT>
__device__ __forceinline__ void ring_issue(unsigned char* smem, const FilterArgs& a, int64_t r0,
                                           bool valid, int c, int sb, int wid, int lane,
                                           __amdgpu_buffer_rsrc_t qr) {
  using L = Lay<XT>;
  const int64_t rows = valid ? (a.n - r0 < kBM ? a.n - r0 : kBM) : 0;
  const __amdgpu_buffer_rsrc_t xr =
      make_rsrc(reinterpret_cast<const XT*>(a.X) + (valid ? r0 : 0) * (int64_t)a.d,
                rows * a.d * (int64_t)sizeof(XT));
  const int k0 = c * kBK;
  unsigned char* st = smem + sb * L::stage;
#pragma unroll
  for (int i = 0; i < L::xdma; ++i) {
    const int j = wid * L::xdma + i;  // 1-KB block of the stage's X image
    if (j >= L::xblocks) {            // wave-uniform: a dummy keeps the count
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_ptr)(smem + L::dummy), 16, 0x7fff0000u,
                                               0, 0, 0);
      continue;
    }
    uint32_t voff;
    if constexpr (sizeof(XT) == 4) {  // 8 rows x 8 pieces of 16 B per block
      const int row = 8 * j + (lane >> 3);
      const int p = (lane & 7) ^ ((row >> 1) & 7);
      voff = k0 + p * 4 < a.d ? (uint32_t)((row * a.d + p * 4) * 4) : 0x7fff0000u;
    } else {  // 16 rows x 4 pieces
      const int row = 16 * j + (lane >> 2);
      const int p = (lane & 3) ^ ((row >> 2) & 3);
      voff = k0 + p * 8 < a.d ? (uint32_t)((row * a.d + p * 8) * 2) : 0x7fff0000u;
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_ptr)(st + j * 1024), 16, voff,
                                             k0 * (int)sizeof(XT), 0, 2 /* nt */);
  }
#pragma unroll
  for (int i = 0; i < L::qdma; ++i) {
    const int j = wid * L::qdma + i;  // 16 queries x 4 pieces per block
    if (j >= L::qblocks) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(qr, (lds_ptr)(smem + L::dummy), 16, 0x7fff0000u,
                                               0, 0, 0);
      continue;
    }
    const int q = 16 * j + (lane >> 2);
    const int p = (lane & 3) ^ ((q >> 2) & 3);
    const uint32_t voff = (uint32_t)(q * 64 + p * 16);  // blocked layout (FilterArgs::Qh)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(qr, (lds_ptr)(st + L::xbytes + j * 1024), 16, voff,
                                             (int)(c * a.qstride * 64), 0, 0);
  }
}

// MFMAs of one stage: 2 k-steps x (2 row tiles x 4 query tiles).  Waves of
// query group 0 also accumulate the rows' sums of squares and fp16-overflow
// flags from the values they read.
// kv = d - (first k of the chunk): elements at k >= d are zeroed (the DMA of a
// piece past the row end is dropped, leaving stale LDS there; the query tile
// is zero-padded, but the row sums must not see it).
template <typename XT, bool IMG>
__device__ __forceinline__ void ring_compute(f32x16 (&acc)[2][kQT], const unsigned char* st,
                                             int rg, int qg, int l32, int h, int kv,
                                             float (&sq)[2], uint32_t& ovf) {
  using L = Lay<XT>;
#pragma unroll
  for (int s = 0; s < kBK / 16; ++s) {
    f16x8 av[2], bv[kQT];
    const int kf = 16 * s + 8 * h;  // first k of this lane's fragment, relative to the chunk
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int R = rg * 64 + t * 32 + l32;
      if constexpr (sizeof(XT) == 4) {
        const int p0 = 4 * s + 2 * h, sw = (R >> 1) & 7;
        f32x4 a0 = *reinterpret_cast<const f32x4*>(st + R * L::xrow + ((p0 ^ sw) * 16));
        f32x4 a1 = *reinterpret_cast<const f32x4*>(st + R * L::xrow + (((p0 + 1) ^ sw) * 16));
        if (kf >= kv) a0 = f32x4(0.f);
        if (kf + 4 >= kv) a1 = f32x4(0.f);
        const f16x4 c0 = __builtin_convertvector(a0, f16x4);
        const f16x4 c1 = __builtin_convertvector(a1, f16x4);
        av[t] = __builtin_shufflevector(c0, c1, 0, 1, 2, 3, 4, 5, 6, 7);
        if (qg == 0) {
          float m = 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sq[t] = fmaf(a0[e], a0[e], sq[t]);
            sq[t] = fmaf(a1[e], a1[e], sq[t]);
            m = fmaxf(m, fmaxf(fabsf(a0[e]), fabsf(a1[e])));
          }
          ovf |= (uint32_t)(m >= 65520.f) << t;
        }
      } else {
        const int p = 2 * s + h;
        av[t] = *reinterpret_cast<const f16x8*>(st + R * L::xrow + ((p ^ ((R >> 2) & 3)) * 16));
        if (kf >= kv) av[t] = f16x8(0);
        if (!IMG && qg == 0) {
#pragma unroll
          for (int e = 0; e < 8; ++e) sq[t] = fmaf((float)av[t][e], (float)av[t][e], sq[t]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kQT; ++u) {
      const int Q = qg * kQT * 32 + u * 32 + l32;
      const int p = 2 * s + h;
      bv[u] = *reinterpret_cast<const f16x8*>(st + L::xbytes + Q * 64 + ((p ^ ((Q >> 2) & 3)) * 16));
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < kQT; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[t], bv[u], acc[t][u], 0, 0, 0);
  }
}

// Wait until this wave's DMAs of the stage to be read have landed (the last
// N issued stay in flight), then the workgroup barrier: every wave's DMAs of
// that stage are in, and every wave is done reading the stage being refilled.
template <int N>
__device__ __forceinline__ void ring_sync() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
}  // namespace ring

// IMG: the rows are an f32 corpus's fp16 filter image (row sums from rowinfo)
template <typename XT, int METRIC, bool IMG>
__global__ void __launch_bounds__(ring::kThreads, ring::kWaves / 4) ring_kernel(FilterArgs a) {
  using namespace ring;
  using L = Lay<XT>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* rinfo = reinterpret_cast<float*>(smem + L::rinfo);
  float* rterm = reinterpret_cast<float*>(smem + L::rterm);
  uint32_t* rflags = reinterpret_cast<uint32_t*>(smem + L::rflags);
  f32x4* qtab = reinterpret_cast<f32x4*>(smem + L::qtab);
  float2* qab = reinterpret_cast<float2*>(smem + L::qab);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR)
  const int rg = wid % kRG, qg = wid / kRG;  // 64-row group, query group
  const int h = lane >> 5, l32 = lane & 31;
  const int64_t q0 = (int64_t)blockIdx.y * kBQ;
  const int nch = (a.d + kBK - 1) / kBK;
  const int diag = a.diag;
  filter_query_table<METRIC>(a, q0, qtab, qab, tid, kThreads);
  const __amdgpu_buffer_rsrc_t qr =
      make_rsrc(a.Qh + q0 * 32, ((int64_t)(a.dq / 32 - 1) * a.qstride + kBQ) * 64);

  // step sequence: (tile ti, chunk c) -> stage buffer (step % 3)
  auto tile_r0 = [&](int64_t ti) -> int64_t { return (a.tile_start + ti * a.tile_stride) * kBM; };
  int64_t ti = blockIdx.x;
  if (ti >= a.num_tiles) return;
  // prologue: steps 0 and 1
  int64_t it = ti;  // tile of the next step to issue
  int ic = 0;       // its chunk
  int isb = 0;      // its stage buffer
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    ring_issue<XT>(smem, a, tile_r0(it), it < a.num_tiles, ic, isb, wid, lane, qr);
    if (++ic == nch) {
      ic = 0;
      it += gridDim.x;
    }
    isb = isb == kStages - 1 ? 0 : isb + 1;
  }
  int sb = 0;  // stage buffer of the current step
  int par = 0;
  for (; ti < a.num_tiles; ti += gridDim.x, par ^= 1) {
    const int64_t r0 = tile_r0(ti);
    uint32_t* flags = rflags + par * kRowFlagWords;
    if (tid < kRowFlagWords) flags[tid] = 0u;  // (read two tiles back; barriers since)
    f32x16 acc[2][kQT];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < kQT; ++u) acc[t][u] = f32x16(0.f);
    float sq[2] = {0.f, 0.f};
    uint32_t ovf = 0u;
    for (int c = 0; c < nch; ++c) {
      ring_sync<L::ndma>();
      ring_issue<XT>(smem, a, tile_r0(it), it < a.num_tiles, ic, isb, wid, (int)opaque(lane), qr);
      if (++ic == nch) {
        ic = 0;
        it += gridDim.x;
      }
      isb = isb == kStages - 1 ? 0 : isb + 1;
      if (!(diag & 4)) {
        const int ol = (int)opaque(lane);
        ring_compute<XT, IMG>(acc, smem + sb * L::stage, rg, qg, ol & 31, ol >> 5, a.d - c * kBK, sq,
                         ovf);
      }
      sb = sb == kStages - 1 ? 0 : sb + 1;
    }
    // row values: query-group-0 waves hold the rows' partial sums (lane halves)
    if (qg == 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        sq[t] += __shfl_xor(sq[t], 32);
        const uint32_t of = (ovf | __shfl_xor(ovf, 32)) >> t & 1u;
        if (h == 0) {
          const int lr = rg * 64 + t * 32 + l32;
          const int64_t row = r0 + lr;
          bool ok = row < a.n;
          if constexpr (IMG) sq[t] = ok ? a.rowinfo[row] : 0.f;
          if (ok && a.mask != nullptr) ok = (a.mask[row >> 5] >> (row & 31)) & 1u;
          float rv;
          if constexpr (METRIC == 0) {
            rv = sq[t];
          } else if constexpr (METRIC == 1) {
            rv = sqrtf(sq[t]);
          } else {
            rv = fmaxf(sqrtf(sq[t]), 1e-12f);
          }
          if (!(sq[t] <= 3.4e38f) || of) rv = __builtin_nanf("");
          filter_note_row<METRIC>(rinfo, rterm, flags, lr, rv, ok);
        }
      }
    }
    lds_sync();
    if (!(diag & 2)) {
      const int ol = (int)opaque(lane);  // keep the epilogue's lane math out of the chunk loop
      filter_epilogue<METRIC, kQT>(acc, rinfo, rterm, flags, qtab, qab, a, q0, r0, rg, qg, ol >> 5,
                                   ol & 31, diag);
    }
  }
  // drain: the ring's last DMAs (empty descriptors past the end) must land
  // before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <typename XT, bool IMG = false>
static int launch_ring(const FilterArgs& a, int metric, hipStream_t stream) {
  const size_t smem = ring::Lay<XT>::total;
  const void* fn = metric == FX_METRIC_COS ? (const void*)ring_kernel<XT, 2, IMG>
                   : metric == FX_METRIC_IP ? (const void*)ring_kernel<XT, 1, IMG>
                                            : (const void*)ring_kernel<XT, 0, IMG>;
  if (int rc = allow_lds(fn)) return rc;
  int cus = 0;
  int rc = device_cus(&cus);
  if (rc) return rc;
  const int64_t qtiles = (a.nq + ring::kBQ - 1) / ring::kBQ;
  int64_t bx = cus;
  if (bx > a.num_tiles) bx = a.num_tiles;
  for (int64_t y0 = 0; y0 < qtiles; y0 += 65535) {
    FilterArgs b = a;
    const int64_t yn = (qtiles - y0) < 65535 ? (qtiles - y0) : 65535;
    b.Qh = a.Qh + y0 * ring::kBQ * 32;
    b.qinfo = a.qinfo + y0 * ring::kBQ * 4;
    b.thr = a.thr + y0 * ring::kBQ;
    b.count = a.count + y0 * ring::kBQ * kCountStride;
    b.cand = a.cand + y0 * ring::kBQ * (int64_t)a.cap;
    if (a.cand_ub) b.cand_ub = a.cand_ub + y0 * ring::kBQ * (int64_t)a.cap;
    b.nq = a.nq - y0 * ring::kBQ;
    void* args[] = {(void*)&b};
    hipError_t e = hipLaunchKernel(fn, dim3((unsigned)bx, (unsigned)yn), dim3(ring::kThreads),
                                   args, smem, stream);
    if (e != hipSuccess) {
      set_error("ring_kernel launch: %s", hipGetErrorString(e));
      return FX_EHIP;
    }
  }
  return check_launch("ring_kernel");
}
#endif  // FX_DIAG_BUILD

int launch(const FilterArgs& a, int metric, hipStream_t stream) {
  if (a.num_tiles <= 0) return FX_OK;
  const bool f16 = a.dtype == FX_DTYPE_F16;
  if (a.rowinfo != nullptr && image_tiled()) {  // the image in MFMA fragment order
#if FX_FILTER_IMG5
    return launch_img5(a, metric, stream);
#elif FX_FILTER_IMG4
    return launch_img4(a, metric, stream);
#elif FX_FILTER_IMG3
#if FX_FILTER_BQ >= 256
    if (img8_serves(a)) return launch_img8(a, metric, stream);
#endif
    return launch_img3(a, metric, stream);
#elif FX_FILTER_IMG2
    return launch_img2(a, metric, stream);
#else
    set_error("filter: the tiled image is not compiled into this variant");
    return FX_EUNSUPPORTED;
#endif
  }
#ifdef FX_DIAG_BUILD
  if (filter_ring()) {
    if (a.rowinfo != nullptr) {
      if (!f16) {
        set_error("filter: a filter image is fp16");
        return FX_EINVAL;
      }
      return launch_ring<_Float16, true>(a, metric, stream);
    }
    return f16 ? launch_ring<_Float16>(a, metric, stream) : launch_ring<float>(a, metric, stream);
  }
#endif
  const size_t smem = sizeof(FilterShared);
  // (the 256-query compilation serves f32 rows, h256 fp16 rows, q64 both)
#if FX_FILTER_ROWS & 1
#define FX_F32_KERNEL(m) (const void*)filter_kernel<float, m, false>
#else
#define FX_F32_KERNEL(m) nullptr
#endif
#if FX_FILTER_ROWS & 2
#define FX_F16_KERNEL(m) (const void*)filter_kernel<_Float16, m, false>
#ifdef FX_DIAG_BUILD  // row-major images (rejected: the tiled image is 7-10 % faster)
#define FX_IMG_KERNEL(m) (const void*)filter_kernel<_Float16, m, true>
#else
#define FX_IMG_KERNEL(m) nullptr
#endif
#else
#define FX_F16_KERNEL(m) nullptr
#define FX_IMG_KERNEL(m) nullptr
#endif
  const void* fns[3][3] = {{FX_F32_KERNEL(0), FX_F32_KERNEL(1), FX_F32_KERNEL(2)},
                           {FX_F16_KERNEL(0), FX_F16_KERNEL(1), FX_F16_KERNEL(2)},
                           {FX_IMG_KERNEL(0), FX_IMG_KERNEL(1), FX_IMG_KERNEL(2)}};
#undef FX_F32_KERNEL
#undef FX_F16_KERNEL
#undef FX_IMG_KERNEL
  const int rt = a.rowinfo != nullptr ? 2 : f16 ? 1 : 0;
  if ((a.rowinfo != nullptr && !f16) || fns[rt][0] == nullptr) {
    set_error("filter: row type not compiled into this variant");
    return FX_EUNSUPPORTED;
  }
  const void* fn = fns[rt][metric == FX_METRIC_COS ? 2 : metric == FX_METRIC_IP ? 1 : 0];
  if (int rc = allow_lds(fn)) return rc;
  int cus = 0;
  int rc = device_cus(&cus);
  if (rc) return rc;
  const int64_t qtiles = (a.nq + fBQ - 1) / fBQ;
  int64_t bx = (int64_t)cus * FX_FILTER_BPC;
  if (bx > a.num_tiles) bx = a.num_tiles;
  for (int64_t y0 = 0; y0 < qtiles; y0 += 65535) {
    FilterArgs b = a;
    const int64_t yn = (qtiles - y0) < 65535 ? (qtiles - y0) : 65535;
    b.Qh = a.Qh + y0 * fBQ * 32;
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

}  // namespace FX_FILTER_IMPL

#ifndef FX_FILTER_VARIANT
namespace q64 {
int launch(const FilterArgs& a, int metric, hipStream_t stream);  // knn_filter_q64.hip
}
namespace q128 {
int launch(const FilterArgs& a, int metric, hipStream_t stream);  // knn_filter_q128.hip
int launch_img6(const FilterArgs& a, int metric, hipStream_t stream);
bool img6_fits(int dq);
}
namespace q64i {  // knn_filter_q64i.hip
int launch(const FilterArgs& a, int metric, hipStream_t stream);
int launch_img6(const FilterArgs& a, int metric, hipStream_t stream);
bool img6_fits(int dq);
}
namespace h256 {
int launch(const FilterArgs& a, int metric, hipStream_t stream);  // knn_filter_h256.hip
}

// The register-staged kernel (measured faster for both row types: 8.5 vs
// 10.1 ms for configs[2]; see DESIGN.md for fp16) and filter images in MFMA
// fragment order (filter_img2_kernel).  Diagnostic builds keep the rejected
// LDS-DMA ring (FX_FILTER_RING=1) and row-major images (FX_IMAGE_TILED=0;
// read when an image is built and when it is searched: both must happen
// under the same setting).
bool image_tiled() { return diag_env("FX_IMAGE_TILED", 1) != 0; }

bool filter_ring() { return diag_env("FX_FILTER_RING", 0) != 0; }

// Batches of <= 64 queries take the 64-query tiles, 65..128 the 128-query ones
// (their Qh is padded to 64 / 128, filter_query_pad)
int launch_filter(const FilterArgs& a, int metric, hipStream_t stream) {
  // int8 images: a batch that fits one resident slice (<= 128 queries) runs
  // filter_img6_kernel (option "img6" 1; configs[1] 1.29 vs 1.34 ms, 128 L2
  // queries 1.81 vs 1.93 ms), larger ones filter_img3_kernel with 256-query
  // tiles (256 cosine queries: 2.97 ms against 3.34 ms for two img6 slices;
  // option 2 forces the slices, 0 disables img6)
  if (a.img8) {
    const int64_t i6 = option(kOptImg6);
    if (a.nq <= 64) {
      if (i6 >= 1 && q64i::img6_fits(a.dq)) return q64i::launch_img6(a, metric, stream);
      return q64i::launch(a, metric, stream);
    }
    if (a.nq <= 128) {
      if (i6 >= 1 && q128::img6_fits(a.dq)) return q128::launch_img6(a, metric, stream);
      return q128::launch(a, metric, stream);
    }
    if (i6 >= 2 && q128::img6_fits(a.dq)) return q128::launch_img6(a, metric, stream);
    return q256::launch(a, metric, stream);
  }
  if (a.nq <= 64) return q64::launch(a, metric, stream);
  if (a.nq <= 128 && !filter_ring()) return q128::launch(a, metric, stream);
  // tiled images: K chunks of 32 (5.07-5.10 vs 5.48-5.49 ms for configs[2]
  // in the 64-wide h256 build, profiles/r02_filter_img_bk32.log)
  if (a.rowinfo != nullptr && image_tiled()) return q256::launch(a, metric, stream);
  if (a.dtype == FX_DTYPE_F16 && !filter_ring()) return h256::launch(a, metric, stream);
  return q256::launch(a, metric, stream);
}

// rows per tile of the kernel launch_filter picks for the dtype (the 64-query
// variant tiles rows like the 256-query one)
int filter_tile_rows(int dtype) {
  (void)dtype;
#ifdef FX_DIAG_BUILD
  static_assert(q256::ring::kBM == q256::fBM, "one tile height for every filter kernel");
#endif
  return q256::fBM;
}

int filter_query_pad(int64_t nq) { return nq <= 64 ? 64 : nq <= 128 && !filter_ring() ? 128 : 256; }
int filter_dq(int d) { return (d + 63) / 64 * 64; }  // covers every variant's K chunk

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
  // blocks of 32 components, query-major inside a block (FilterArgs::Qh):
  // a K chunk of a query tile is one contiguous run of whole cache lines
  _Float16* out = reinterpret_cast<_Float16*>(Qh) + q * 32;
  auto at = [&](int i) -> _Float16& { return out[(int64_t)(i >> 5) * nq_pad * 32 + (i & 31)]; };
  if (q >= nq) {
    for (int i = lane; i < dq; i += 64) at(i) = (_Float16)0.f;
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
  for (int i = lane; i < dq; i += 64) at(i) = (_Float16)(i < d ? qv[i] * scale : 0.f);
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

// The fp16 filter image of an f32 corpus (fx_filter_image): every component
// converted exactly as the f32 filter converts it in registers (round to
// nearest even), plus per row the f32 sum of squares of the original
// components, NaN when the row must be forced through (non-finite, or a
// component >= 65520 that becomes an fp16 infinity).  The filter then streams
// 2 bytes per component instead of 4 and skips its in-loop conversion and row
// sums; candidates are still rescored from the f32 rows, so results do not
// change.  One wave per row, grid-stride.
typedef float img_f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 img_f16x4 __attribute__((ext_vector_type(4)));
#ifdef FX_DIAG_BUILD  // row-major images (FX_IMAGE_TILED=0)
__global__ void __launch_bounds__(256) image_kernel(const float* __restrict__ X, int64_t n, int d,
                                                    _Float16* __restrict__ img,
                                                    float* __restrict__ rowinfo) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += nw) {
    const img_f32x4* xr = reinterpret_cast<const img_f32x4*>(X + r * d);
    img_f16x4* ir = reinterpret_cast<img_f16x4*>(img + r * d);
    float s = 0.f, m = 0.f;
    for (int i = lane; i < d / 4; i += 64) {
      const img_f32x4 v = __builtin_nontemporal_load(xr + i);
      ir[i] = __builtin_convertvector(v, img_f16x4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s = fmaf(v[e], v[e], s);
        m = fmaxf(m, fabsf(v[e]));
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      s += __shfl_xor(s, o);
      m = fmaxf(m, __shfl_xor(m, o));
    }
    if (lane == 0) rowinfo[r] = (s <= 3.4e38f && m < 65520.f) ? s : __builtin_nanf("");
  }
}
#endif  // FX_DIAG_BUILD

// The image in MFMA fragment order (FX_IMAGE_TILED): one wave per 32-row
// tile, grid-stride.  Each k-step, lane l reads components 16 s + 8 (l / 32)
// .. + 7 of row 32 t + l % 32 (two 16-B loads; the other half of each line is
// read by the next k-step, from L2) and the wave writes the k-step's KB of
// the image as one contiguous store.  Padding rows and components are written
// as zeros (no memset).  d % 8 == 0 (fx_filter_image checks).
typedef _Float16 img_f16x8 __attribute__((ext_vector_type(8)));
__global__ void __launch_bounds__(256) image_tiled_kernel(const float* __restrict__ X, int64_t n,
                                                          int d, _Float16* __restrict__ img,
                                                          float* __restrict__ rowinfo) {
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int64_t nt = (n + 31) / 32;
  const int ksteps = (d + 15) / 16;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t < nt; t += nw) {
    const int64_t r = t * 32 + (lane & 31);
    const bool live = r < n;
    const float* xr = X + (live ? r : 0) * (int64_t)d;
    img_f16x8* out = reinterpret_cast<img_f16x8*>(img) + t * ksteps * 64 + lane;
    float s = 0.f, m = 0.f;
#pragma unroll 4
    for (int ks = 0; ks < ksteps; ++ks) {
      // loads without a branch (several k-steps in flight): padding reads a
      // valid address and is zeroed after
      const int k0 = 16 * ks + 8 * h;
      const bool ok = live && k0 < d;
      const float* p = xr + (k0 < d ? k0 : 0);
      // (plain loads: the line's other half is read at the next k-step, from L2;
      // nontemporal loads had it refetched, 2x the bytes)
      img_f32x4 a = *reinterpret_cast<const img_f32x4*>(p);
      img_f32x4 b = *reinterpret_cast<const img_f32x4*>(p + 4);
      if (!ok) {
        a = img_f32x4(0.f);
        b = img_f32x4(0.f);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s = fmaf(a[e], a[e], s);
        s = fmaf(b[e], b[e], s);
        m = fmaxf(m, fmaxf(fabsf(a[e]), fabsf(b[e])));
      }
      const img_f16x4 ca = __builtin_convertvector(a, img_f16x4);
      const img_f16x4 cb = __builtin_convertvector(b, img_f16x4);
      out[ks * 64] = __builtin_shufflevector(ca, cb, 0, 1, 2, 3, 4, 5, 6, 7);
    }
    s += __shfl_xor(s, 32);
    m = fmaxf(m, __shfl_xor(m, 32));
    if (h == 0 && live) rowinfo[r] = (s <= 3.4e38f && m < 65520.f) ? s : __builtin_nanf("");
  }
}

int launch_image(const float* X, int64_t n, int d, void* img, float* rowinfo,
                 hipStream_t stream) {
  if (n <= 0) return FX_OK;
  int cus = 0;
  int rc = device_cus(&cus);
  if (rc) return rc;
  if (image_tiled()) {
    int64_t blocks = ((n + 31) / 32 + 3) / 4;
    if (blocks > (int64_t)cus * 8) blocks = (int64_t)cus * 8;
    hipLaunchKernelGGL(image_tiled_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, X, n, d,
                       reinterpret_cast<_Float16*>(img), rowinfo);
    return check_launch("image_tiled_kernel");
  }
#ifdef FX_DIAG_BUILD
  int64_t blocks = (n + 3) / 4;
  if (blocks > (int64_t)cus * 32) blocks = (int64_t)cus * 32;
  hipLaunchKernelGGL(image_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, X, n, d,
                     reinterpret_cast<_Float16*>(img), rowinfo);
  return check_launch("image_kernel");
#else
  return FX_EUNSUPPORTED;  // (unreachable: image_tiled() is constant)
#endif
}

// ---- int8 filter image (filter_img3_kernel<METRIC, true>; the bounds are
// derived above filter_img3_kernel).  Rows and queries are scaled so that
// their integer images have norm <= 2048 (|x~ . q~| <= 2^22):
//   s = max(max|x| / 127, |x| / (2046 - sqrt(d) / 2)).
__device__ __forceinline__ float i8_norm_cap(int d) { return 2046.f - 0.5f * sqrtf((float)d); }

typedef float img_f32x16 __attribute__((ext_vector_type(16)));

// The image in MFMA fragment order: [ceil(n / 32) row tiles][ceil(d / 32)
// k-steps][64 lanes][16 B]: lane l holds components 32 s + 16 (l / 32) .. + 15
// of row 32 t + l % 32 (the v_mfma_i32_32x32x32_i8 A operand), and per row
// {omega = w + kappa v, 1/s, N/s, n^2/s} (NaN omega: forced).  One wave per
// 32-row tile: a pass for max |x| and n^2, a pass that quantizes, writes and
// accumulates the residual (|x - s x~|^2 in f32 with (d + 8) u slack) and
// w^2 (exact in integers).  d % 8 == 0 (fx_filter_image8 checks).
// T: the corpus's value type, float or _Float16 (the values are the same
// reals in f32, so the bounds below are unchanged; the candidates are rescored
// from the T rows in the scan's order)
// Image row r holds corpus row perm_row(pa, n, r) (image8_perm): the tile's
// 32 rows come from 32 places of the corpus, each still read as whole
// 128-B lines.
template <typename T>
__global__ void __launch_bounds__(256) image8_kernel(const T* __restrict__ X, int64_t n, int d,
                                                    int8_t* __restrict__ img,
                                                    float* __restrict__ rowinfo, uint64_t pa) {
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int64_t nt = (n + 31) / 32;
  const int ksteps = (d + 31) / 32;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const float u = 5.9604644775390625e-08f;
  for (int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t < nt; t += nw) {
    const int64_t r = t * 32 + (lane & 31);
    const bool live = r < n;
    const T* xr = X + (live ? (int64_t)perm_row(pa, n, r) : 0) * (int64_t)d;
    auto load = [&](int ks) {  // components 32 ks + 16 h .. + 15 (zeros past d)
      img_f32x16 v;
      const int k0 = 32 * ks + 16 * h;
      if constexpr (sizeof(T) == 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = k0 + 4 * j;
          const img_f32x4 q4 = (live && k < d) ? *reinterpret_cast<const img_f32x4*>(xr + k)
                                                : img_f32x4(0.f);
          v[4 * j] = q4[0];
          v[4 * j + 1] = q4[1];
          v[4 * j + 2] = q4[2];
          v[4 * j + 3] = q4[3];
        }
      } else {  // 8 halves per 16-B load (d % 8 == 0)
        typedef _Float16 img_f16x8 __attribute__((ext_vector_type(8)));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int k = k0 + 8 * j;
          const img_f16x8 h8 = (live && k < d) ? *reinterpret_cast<const img_f16x8*>(xr + k)
                                                : img_f16x8((_Float16)0.f);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[8 * j + e] = (float)h8[e];
        }
      }
      return v;
    };
    float m = 0.f, n2 = 0.f;
    for (int ks = 0; ks < ksteps; ++ks) {
      const img_f32x16 v = load(ks);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        n2 = fmaf(v[e], v[e], n2);
        m = fmaxf(m, fabsf(v[e]));
      }
    }
    n2 += __shfl_xor(n2, 32);
    m = fmaxf(m, __shfl_xor(m, 32));
    const bool finite = m <= 3.4e38f && n2 <= 3.4e38f;
    const float nrm = sqrtf(n2);
    float sc = fmaxf(m * (1.f / 127.f), nrm / i8_norm_cap(d));
    if (!(sc > 1e-30f) || !finite) sc = 1.f;  // zero / tiny / non-finite rows (forced below)
    const float is = 1.f / sc;
    int w2 = 0;
    float e2 = 0.f;
    int8_t* out = img + (t * ksteps) * 1024 + lane * 16;
    for (int ks = 0; ks < ksteps; ++ks) {
      const img_f32x16 v = load(ks);
      int32_t packed[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t word = 0u;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const float x = v[4 * j + b];
          float qf = rintf(x * is);
          qf = fminf(fmaxf(qf, -127.f), 127.f);
          if (!finite) qf = 0.f;
          const int qi = (int)qf;
          w2 += qi * qi;
          const float res = fmaf(-sc, qf, x);
          e2 = fmaf(res, res, e2);
          word |= ((uint32_t)qi & 0xffu) << (8 * b);
        }
        packed[j] = (int32_t)word;
      }
      *reinterpret_cast<int4*>(out + ks * 1024) = make_int4(packed[0], packed[1], packed[2], packed[3]);
    }
    w2 += __shfl_xor(w2, 32);
    e2 += __shfl_xor(e2, 32);
    if (h == 0 && live) {
      const float e = sqrtf(e2 * (1.f + 2.f * (float)(d + 8) * u)) * (1.f + 4.f * u);
      const float w = sqrtf((float)w2) * (1.f + 2.f * u);
      const float v = e * is * (1.f + 4.f * u);
      float om = (w + kI8Kappa * v) * (1.f + 4.f * u);
      const bool tiny = !(m == 0.f) && !(fmaxf(m * (1.f / 127.f), nrm / i8_norm_cap(d)) > 1e-30f);
      if (!finite || tiny || w > 2048.f || !(om <= 3.4e38f)) om = __builtin_nanf("");
      const float nn = fmaxf(nrm, 1e-12f);
      img_f32x4 info = {om, is, nn * is, n2 * is};
      *reinterpret_cast<img_f32x4*>(rowinfo + r * kI8RowInfo) = info;
    }
  }
}

static uint64_t gcd64(uint64_t a, uint64_t b) {
  while (b != 0) {
    const uint64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

uint64_t image8_perm(int64_t n) {
  if (n <= 2) return 1;
  uint64_t a = (uint64_t)((double)n * 0.6180339887498949) | 1u;
  while (gcd64(a, (uint64_t)n) != 1) a += 2;
  return a % (uint64_t)n;
}

// One workgroup per query (launch_overflow_gate, fx_internal.h), 8 loads in
// flight per thread (k = 1 000: ~50 K F1 candidates per query, 63 -> ~10 us)
constexpr int kGateThreads = 1024;
__global__ void __launch_bounds__(kGateThreads) overflow_gate_kernel(
    const uint64_t* __restrict__ cand, uint32_t* __restrict__ count,
    const uint64_t* __restrict__ thr, int cap, int64_t num, int64_t den) {
  const int64_t q = blockIdx.x;
  __shared__ uint32_t tot;
  const uint32_t c = count[q * kCountStride];
  if (c > (uint32_t)cap) return;  // (already overflowing: recomputed anyway)
  if (threadIdx.x == 0) tot = 0u;
  __syncthreads();
  const uint32_t t = (uint32_t)(thr[q] >> 32);
  const uint64_t* cq = cand + q * (int64_t)cap;
  uint32_t mine = 0u;
  for (uint32_t b = threadIdx.x; b < c; b += kGateThreads * 8) {
    uint64_t e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i = b + j * kGateThreads;
      e[j] = i < c ? cq[i] : kEmpty;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) mine += b + j * kGateThreads < c && (uint32_t)(e[j] >> 32) <= t;
  }
  for (int o = 32; o >= 1; o >>= 1) mine += __shfl_xor(mine, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(&tot, mine);
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t predicted = (uint64_t)c + ((uint64_t)tot * (uint64_t)num + (uint64_t)den - 1) /
                                                 (uint64_t)den;
    if (predicted > (uint64_t)cap) count[q * kCountStride] = (uint32_t)cap + 1u;
  }
}

int launch_overflow_gate(const uint64_t* cand, uint32_t* count, const uint64_t* thr, int64_t nq,
                         int cap, int64_t num, int64_t den, hipStream_t stream) {
  if (nq <= 0) return FX_OK;
  if (nq > 0x7fffffffll || den <= 0) {
    set_error("overflow gate: nq=%lld den=%lld", (long long)nq, (long long)den);
    return FX_EINVAL;
  }
  hipLaunchKernelGGL(overflow_gate_kernel, dim3((unsigned)nq), dim3(kGateThreads), 0, stream, cand,
                     count, thr, cap, num, den);
  return check_launch("overflow_gate_kernel");
}

int launch_image8(const void* X, int dtype, int64_t n, int d, void* img, float* rowinfo,
                  hipStream_t stream) {
  if (n <= 0) return FX_OK;
  int cus = 0;
  int rc = device_cus(&cus);
  if (rc) return rc;
  int64_t blocks = ((n + 31) / 32 + 3) / 4;
  if (blocks > (int64_t)cus * 8) blocks = (int64_t)cus * 8;
  const uint64_t pa = image8_perm(n);
  if (dtype == FX_DTYPE_F16)
    hipLaunchKernelGGL(image8_kernel<_Float16>, dim3((unsigned)blocks), dim3(256), 0, stream,
                       reinterpret_cast<const _Float16*>(X), n, d, reinterpret_cast<int8_t*>(img),
                       rowinfo, pa);
  else
    hipLaunchKernelGGL(image8_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, stream,
                       reinterpret_cast<const float*>(X), n, d, reinterpret_cast<int8_t*>(img),
                       rowinfo, pa);
  return check_launch("image8_kernel");
}

// Per query (one wave): q~ = rint(q / s_q) in int8, zero-padded to dq, in
// 64-component chunks, query-major inside a chunk (chunk c of query q: 64 B
// at (c * nq_pad + q) * 64), and {s_q, R', n_q^2, |q|} with
// R' = max(R, P / kappa) (see "int8 filter image"); sums in double (products
// of f32 and of f32 x int8 are exact there).  A non-finite query, or one whose
// integer image exceeds norm 2048: R' = +inf (forced).
__global__ void qprep8_kernel(const float* __restrict__ Q, int64_t nq, int64_t nq_pad, int d,
                              int dq, int metric, int8_t* __restrict__ Qb,
                              float* __restrict__ qinfo, uint64_t* __restrict__ thr,
                              uint32_t* __restrict__ count) {
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (q >= nq_pad) return;
  if (q < nq && lane == 0) {  // (the search's threshold and append count, when given)
    if (thr != nullptr) thr[q] = ~0ull;
    if (count != nullptr) count[q * kCountStride] = 0u;
  }
  auto at = [&](int i) -> int8_t& {
    return Qb[((int64_t)(i >> 6) * nq_pad + q) * 64 + (i & 63)];
  };
  if (q >= nq) {
    for (int i = lane; i < dq; i += 64) at(i) = 0;
    return;
  }
  const float* qv = Q + q * (int64_t)d;
  double s2 = 0.0;
  float m = 0.f;
  for (int i = lane; i < d; i += 64) {
    s2 = fma((double)qv[i], (double)qv[i], s2);
    m = fmaxf(m, fabsf(qv[i]));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    s2 += __shfl_xor(s2, o);
    m = fmaxf(m, __shfl_xor(m, o));
  }
  const bool finite = m <= 3.4e38f && s2 <= 1e76;
  const double nq_ = sqrt(s2);
  float sc = fmaxf(m * (1.f / 127.f), (float)(nq_ / (double)i8_norm_cap(d)) * (1.f + 1e-6f));
  const bool tiny = m != 0.f && !(sc > 1e-30f);
  if (!(sc > 1e-30f) || !finite) sc = 1.f;
  const float is = 1.f / sc;
  double e2 = 0.0;
  int w2 = 0;
  for (int i = lane; i < dq; i += 64) {
    int qi = 0;
    if (i < d && finite) {
      float qf = rintf(qv[i] * is);
      qf = fminf(fmaxf(qf, -127.f), 127.f);
      qi = (int)qf;
      const double r = (double)qv[i] - (double)sc * (double)qi;  // exact
      e2 = fma(r, r, e2);
    }
    w2 += qi * qi;
    at(i) = (int8_t)qi;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    e2 += __shfl_xor(e2, o);
    w2 += __shfl_xor(w2, o);
  }
  if (lane == 0) {
    const double u = 5.9604644775390625e-08;
    const double g = (double)(d + 2) * u * 1.01;
    const double eq = sqrt(e2) * (1.0 + 1e-12);
    double P = nq_ / sc, R = eq / sc;
    if (metric == FX_METRIC_IP) {
      R += g * nq_ / sc;
      P *= 1.0 + g;
    }
    double rp = R > P / (double)kI8Kappa ? R : P / (double)kI8Kappa;
    rp *= 1.0 + 1e-6;
    if (!finite || tiny || sqrt((double)w2) > 2048.0) rp = __builtin_inf();
    float* info = qinfo + q * kI8QInfo;
    info[0] = sc;
    info[1] = __double2float_ru(rp);
    info[2] = (float)s2;
    info[3] = (float)nq_;
  }
}

int launch_qprep8(const float* Q, int64_t nq, int64_t nq_pad, int d, int dq, int metric,
                  int8_t* Qb, float* qinfo, hipStream_t stream, uint64_t* thr, uint32_t* count) {
  hipLaunchKernelGGL(qprep8_kernel, dim3((unsigned)((nq_pad + 3) / 4)), dim3(256), 0, stream, Q,
                     nq, nq_pad, d, dq, metric, Qb, qinfo, thr, count);
  return check_launch("qprep8_kernel");
}

#endif  // FX_FILTER_VARIANT

}  // namespace fx
