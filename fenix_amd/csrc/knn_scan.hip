// Fused distance scan + per-wave top-k for one corpus shard, gfx950.
//
// Replaces, for the brute-force branch of io.index.call (coding=None):
//   src/fenix/io/index/index.py:137-162  per-Arrow-chunk scalar UDF that calls
//   src/fenix/io/coder/coder.py:38-50    torch.cdist / -u@v / cosine on CPU,
//   src/fenix/io/index/index.py:165-168  then pc.select_k_unstable over all rows.
//
// Design: the scan is HBM-bound (0.5 flop/byte for one query),
// so one pass over the row-major corpus with 16-byte loads, f32 accumulation
// and a register/LDS-resident query; no GEMM reshaping.  A 64-lane wavefront
// works on 4 rows at a time: lane group g = lane>>4 owns one row and its 16
// lanes read 256 contiguous bytes of that row per load instruction (two full
// 128-B lines), so every load instruction is fully coalesced.  The 16 partial
// sums of a row are folded with 4 DPP row-ops (no LDS traffic).
//
// Top-k is fused: each wavefront keeps its candidates in an LDS list of `cap`
// 64-bit composites (order_key(dist)<<32 | global_row, see fx_common.h) and a
// wave-uniform threshold (the current k-th best).  Rows that cannot enter the
// top-k are rejected with one compare; when the list fills, a wave-local
// 8-bit radix select finds the k-th composite and compacts in place.  At the
// end each wave writes its k best to global memory; knn_merge.hip reduces
// those lists to the final sorted top-k.  No barriers in the main loop.
#include <stdlib.h>

#include "fx_internal.h"
#include "fx_select.h"

// Rows in flight per 16-lane group (U) for each slot count L (slots of 16 B
// per lane per row pass).  Tuning knobs for tools/microbench.py variant builds.
#ifndef FX_U1
#define FX_U1 8
#endif
#ifndef FX_U2
#define FX_U2 2
#endif
#ifndef FX_U3
#define FX_U3 2
#endif
#ifndef FX_U4
#define FX_U4 1
#endif
#ifndef FX_U6
#define FX_U6 1
#endif
#ifndef FX_U8
#define FX_U8 1
#endif
#ifndef FX_U12
#define FX_U12 2  // 768-d f32 / 1536-d f16: 4.40 vs 4.54 ms (interleaved, 10M x 768)
#endif

// Rows in flight per group for quint8 rows (separately tunable).  Converted
// codes take 4x their bytes in registers, so fewer rows per group and more
// waves win: at 768-d (L = 3) U = 1 with 3 blocks/CU runs 1.77 ms vs 2.01 ms
// for U = 2 with 2 (10M rows); U = 4 spills (13.9 ms).
#ifndef FX_Q1
#define FX_Q1 8
#endif
#ifndef FX_Q2
#define FX_Q2 2
#endif
#ifndef FX_Q3
#define FX_Q3 1
#endif
#ifndef FX_Q4
#define FX_Q4 1
#endif
#ifndef FX_Q6
#define FX_Q6 1
#endif
#ifndef FX_Q8
#define FX_Q8 1
#endif
#ifndef FX_Q12
#define FX_Q12 1
#endif

// quint8 rows through a per-wave LDS-DMA ring (global_load_lds): rows in
// flight cost no registers, so more of them stay in flight than the register
// tiles allow.  Rows per lane group per tile and ring depth (tiles):
#ifndef FX_Q8DMA_U
#define FX_Q8DMA_U 1
#endif
#ifndef FX_Q8DMA_AUX  // cache policy of the code stream's LDS-DMA loads (2: nontemporal)
#define FX_Q8DMA_AUX 2
#endif
#ifndef FX_Q8DMA_STAGES
#define FX_Q8DMA_STAGES 3
#endif

namespace fx {

// ---------------------------------------------------------------- helpers --

template <typename T, int W>
struct VecT {
  typedef T type __attribute__((ext_vector_type(W)));
};
template <typename T>
struct VecT<T, 1> {
  typedef T type;
};

template <int W, typename V>
__device__ __forceinline__ float elem(const V& v, int e) {
  if constexpr (W == 1) {
    return (float)v;
  } else {
    return (float)v[e];
  }
}

template <typename V>
__device__ __forceinline__ V load_stream(const V* p) {
#if FX_NONTEMPORAL
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}

// k-th smallest (1-indexed) composite among buf[0..cnt), cnt >= k >= 1.
// Also returns how many entries equal to the k-th belong to the k smallest
// (only the empty sentinel can repeat: real composites carry unique rows).
__device__ uint64_t wave_select(const uint64_t* buf, int cnt, int k, uint32_t* hist, int lane,
                                int* quota_eq) {
  uint64_t prefix = 0, pmask = 0;
  uint32_t need = (uint32_t)k;
  // start at the highest byte in which the entries differ
  uint64_t v_or = 0, v_and = ~0ull;
  for (int i = lane; i < cnt; i += kWave) {
    const uint64_t e = buf[i];
    v_or |= e;
    v_and &= e;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    v_or |= shfl_xor_u64(v_or, m);
    v_and &= shfl_xor_u64(v_and, m);
  }
  const uint64_t diff = v_or ^ v_and;
  const int start = diff ? (63 - __clzll((long long)diff)) / 8 * 8 : 0;
  // the bytes above `start` are common to every entry: they seed the prefix
  pmask = start >= 56 ? 0ull : (~0ull << (start + 8));
  prefix = v_and & pmask;
  for (int shift = start; shift >= 0; shift -= 8) {
    for (int i = lane; i < 256; i += kWave) hist[i] = 0u;
    wave_sync();
    for (int base = 0; base < cnt; base += kWave) {
      const int i = base + lane;
      const uint64_t e = i < cnt ? buf[i] : kEmpty;
      hist_add(hist, (uint32_t)(e >> shift) & 255u, i < cnt && (e & pmask) == prefix);
    }
    wave_sync();
    uint32_t h0 = hist[4 * lane + 0], h1 = hist[4 * lane + 1];
    uint32_t h2 = hist[4 * lane + 2], h3 = hist[4 * lane + 3];
    uint32_t s = h0 + h1 + h2 + h3;
    uint32_t incl = wave_incl_scan(s, lane), excl = incl - s;
    bool here = excl < need && need <= incl;
    uint64_t bb = __ballot(here);
    int src = __ffsll((unsigned long long)bb) - 1;
    uint32_t digit = 0, below = 0, inbin = 0;
    if (here) {
      uint32_t c = excl;
      if (c + h0 >= need) {
        digit = 4 * lane; below = c; inbin = h0;
      } else if (c + h0 + h1 >= need) {
        digit = 4 * lane + 1; below = c + h0; inbin = h1;
      } else if (c + h0 + h1 + h2 >= need) {
        digit = 4 * lane + 2; below = c + h0 + h1; inbin = h2;
      } else {
        digit = 4 * lane + 3; below = c + h0 + h1 + h2; inbin = h3;
      }
    }
    digit = __shfl(digit, src);
    below = __shfl(below, src);
    inbin = __shfl(inbin, src);
    need -= below;
    prefix |= (uint64_t)digit << shift;
    pmask |= 0xffull << shift;
    if (inbin == need) {
      // the whole bucket is inside the k smallest: the k-th is its maximum
      uint64_t m = 0;
      for (int i = lane; i < cnt; i += kWave) {
        uint64_t e = buf[i];
        if ((e & pmask) == prefix && e > m) m = e;
      }
      m = wave_max_u64(m);
      int eq = 0;
      for (int i = lane; i < cnt; i += kWave) eq += (buf[i] == m) ? 1 : 0;
      *quota_eq = wave_sum_i(eq);
      wave_sync();
      return m;
    }
    wave_sync();
  }
  *quota_eq = (int)need;
  return prefix;
}

// In-place, order-preserving compaction of buf[0..cnt) to the entries < T
// plus the first quota_eq entries == T.  Returns the new count.
__device__ int wave_compact(uint64_t* buf, int cnt, uint64_t T, int quota_eq, int lane) {
  const uint64_t ltmask = (1ull << lane) - 1ull;
  int w = 0, eqk = 0;
  for (int base = 0; base < cnt; base += kWave) {
    int i = base + lane;
    bool in = i < cnt;
    uint64_t e = in ? buf[i] : kEmpty;
    bool lt = in && e < T;
    bool eq = in && e == T;
    uint64_t beq = __ballot(eq);
    bool keep = lt || (eq && eqk + __popcll(beq & ltmask) < quota_eq);
    eqk += __popcll(beq);
    uint64_t bk = __ballot(keep);
    if (keep) buf[w + __popcll(bk & ltmask)] = e;
    w += __popcll(bk);
  }
  wave_sync();
  return w;
}

// ------------------------------------------------------------ scan kernel --
//
// T: element type (float / _Float16); W: elements per 16-B (or scalar) slot;
// L: slots per lane per row pass (the row covers 16*L slots per pass, more
// passes if the row is longer); U: rows per lane group per tile.
//
// Software pipeline: while a wave reduces tile i it already has tile i+1's
// loads in flight (two register tiles, the loop unrolled by two so no moves),
// so every wave keeps HBM requests outstanding continuously instead of
// alternating load bursts with compute.

template <typename T, int W, int L, int U>
struct RowTile {
  typename VecT<T, W>::type v[U][L];
  int64_t row[U];  // position in the scanned range (list index with a row list)
  int64_t src[U];  // corpus row (== row without a row list)
  bool valid[U];
};

struct ScanCtx {
  const ScanArgs* a;
  const float* q_lds;
  uint64_t* buf;
  uint32_t* hist;
  int S, lane, grp, jl, qi;
  int64_t hi;
  float qnorm;
  float qscale, qshift;  // uint8 codes: dequantised in registers
  bool topk;
};

template <typename T, int W, int L, int U>
__device__ __forceinline__ void tile_load(RowTile<T, W, L, U>& t, int64_t it, int ch,
                                          const ScanCtx& c) {
  using V = typename VecT<T, W>::type;
  const ScanArgs& a = *c.a;
  const T* X = reinterpret_cast<const T*>(a.X);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    t.row[u] = it + u * 4 + c.grp;
    t.valid[u] = t.row[u] < c.hi;
    t.src[u] = t.row[u];
    if (a.rows != nullptr && t.valid[u]) t.src[u] = a.rows[t.row[u]];
    if (a.mask != nullptr && t.valid[u])
      t.valid[u] = (a.mask[t.src[u] >> 5] >> (t.src[u] & 31)) & 1u;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const V* rp = reinterpret_cast<const V*>(X + t.src[u] * (int64_t)a.d);
#pragma unroll
    for (int cc = 0; cc < L; ++cc) {
      const int s = ch * 16 * L + cc * 16 + c.jl;
      if (t.valid[u] && s < c.S) {
        t.v[u][cc] = load_stream(rp + s);
      } else if constexpr (sizeof(T) == 1) {
        t.v[u][cc] = V((T)c.qshift);  // the zero-point code dequantises to exactly 0
      } else {
        t.v[u][cc] = V(0);
      }
    }
  }
}

template <typename T, int W, int L, int U, int METRIC>
__device__ __forceinline__ void tile_accumulate(const RowTile<T, W, L, U>& t, int ch,
                                                const ScanCtx& c, float (&acc)[U],
                                                float (&acc2)[U]) {
  if constexpr (sizeof(T) == 1) {
    // quint8 codes, value = qscale * (code - qshift).  Per element: one
    // ubyte->f32 convert and packed fp32 ops on pairs (v_pk_add/v_pk_fma):
    //   L2   d = code - q'  with q' = qshift + q/qscale (query pre-transformed
    //        in LDS), sum d^2;  distance = qscale * sqrt(sum)
    //   IP   sum (code - qshift) q;            distance = -qscale * sum
    //   cos  sum (code - qshift) q and (code - qshift)^2, scaled in tile_finish
    // (vs dequantise-then-compute: 2-2.5 VALU ops per byte instead of 5-6; the
    // scan was VALU-bound at 3.6 TB/s).
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef float f16v __attribute__((ext_vector_type(16)));
    static_assert(W == 16 || W == 1, "quint8 rows are scanned 16 codes per lane");
    const f2 z2 = {c.qshift, c.qshift};
#pragma unroll
    for (int cc = 0; cc < L; ++cc) {
      const int s = ch * 16 * L + cc * 16 + c.jl;
      if constexpr (W == 1) {
        const float qv = c.q_lds[s];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const float x = (float)t.v[u][cc];
          if constexpr (METRIC == 0) {
            const float d = x - qv;
            acc[u] = fmaf(d, d, acc[u]);
          } else {
            const float d = x - c.qshift;
            acc[u] = fmaf(d, qv, acc[u]);
            if constexpr (METRIC == 2) acc2[u] = fmaf(d, d, acc2[u]);
          }
        }
      } else {
        f2 q2[8];
        const f2* qp = reinterpret_cast<const f2*>(c.q_lds + s * W);
#pragma unroll
        for (int p = 0; p < 8; ++p) q2[p] = qp[p];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const f16v xf = __builtin_convertvector(t.v[u][cc], f16v);
          f2 a2 = {0.f, 0.f}, b2 = {0.f, 0.f};
#pragma unroll
          for (int p = 0; p < 8; ++p) {
            const f2 x2 = {xf[2 * p], xf[2 * p + 1]};
            if constexpr (METRIC == 0) {
              const f2 d = x2 - q2[p];
              a2 = __builtin_elementwise_fma(d, d, a2);
            } else {
              const f2 d = x2 - z2;
              a2 = __builtin_elementwise_fma(d, q2[p], a2);
              if constexpr (METRIC == 2) b2 = __builtin_elementwise_fma(d, d, b2);
            }
          }
          acc[u] += a2.x + a2.y;
          if constexpr (METRIC == 2) acc2[u] += b2.x + b2.y;
        }
      }
    }
    return;
  }
#pragma unroll
  for (int cc = 0; cc < L; ++cc) {
    const int s = ch * 16 * L + cc * 16 + c.jl;
    float qv[W];
#pragma unroll
    for (int e = 0; e < W; ++e) qv[e] = c.q_lds[s * W + e];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int e = 0; e < W; ++e) {
        const float x = elem<W>(t.v[u][cc], e);
        if constexpr (METRIC == 0) {
          const float d = x - qv[e];
          acc[u] = fmaf(d, d, acc[u]);
        } else if constexpr (METRIC == 1) {
          acc[u] = fmaf(x, qv[e], acc[u]);
        } else {
          acc[u] = fmaf(x, qv[e], acc[u]);
          acc2[u] = fmaf(x, x, acc2[u]);
        }
      }
    }
  }
}

// Distances of the tile's rows -> output (distance mode) or candidate list.
template <typename T, int W, int L, int U, int METRIC>
__device__ __forceinline__ void tile_finish(const RowTile<T, W, L, U>& t, float (&acc)[U],
                                            float (&acc2)[U], const ScanCtx& c, uint64_t& thr,
                                            int& cnt) {
  const ScanArgs& a = *c.a;
  float dist[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const float s1 = sum16(acc[u]);
    if constexpr (sizeof(T) == 1) {  // quint8: sums are in code units
      if constexpr (METRIC == 0) {
        dist[u] = c.qscale * sqrtf(s1);
      } else if constexpr (METRIC == 1) {
        dist[u] = -(c.qscale * s1);
      } else {
        const float s2 = sum16(acc2[u]);
        const float nx = fmaxf(c.qscale * sqrtf(s2), 1e-12f);
        dist[u] = 0.5f - 0.5f * ((c.qscale * s1) / (nx * c.qnorm));
      }
    } else if constexpr (METRIC == 0) {
      dist[u] = sqrtf(s1);
    } else if constexpr (METRIC == 1) {
      dist[u] = -s1;
    } else {
      const float s2 = sum16(acc2[u]);
      const float nx = fmaxf(sqrtf(s2), 1e-12f);
      dist[u] = 0.5f - 0.5f * (s1 / (nx * c.qnorm));
    }
  }
  if (!c.topk) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (c.jl == 0 && t.row[u] < c.hi)
        a.out_dist[(size_t)c.qi * a.n + t.row[u]] = t.valid[u] ? dist[u] : __builtin_nanf("");
    }
    return;
  }
  const uint64_t ltmask = (1ull << c.lane) - 1ull;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t comp = make_comp(dist[u], (uint32_t)(a.row_base + t.src[u]));
    const bool p = (c.jl == 0) && t.valid[u] && comp < thr;
    const uint64_t b = __ballot(p);
    if (b) {
      if (p) c.buf[cnt + __popcll(b & ltmask)] = comp;
      cnt += __popcll(b);
    }
  }
  if (cnt > a.cap - 4 * U) {
    wave_sync();
    int quota;
    thr = wave_select(c.buf, cnt, a.k, c.hist, c.lane, &quota);
    cnt = wave_compact(c.buf, cnt, thr, quota, c.lane);
  }
}

template <typename T, int W, int L, int U, int METRIC>
__device__ __forceinline__ void tile_consume(const RowTile<T, W, L, U>& t, const ScanCtx& c,
                                             uint64_t& thr, int& cnt) {
  float acc[U], acc2[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = acc2[u] = 0.f;
  tile_accumulate<T, W, L, U, METRIC>(t, 0, c, acc, acc2);
  tile_finish<T, W, L, U, METRIC>(t, acc, acc2, c, thr, cnt);
}

#ifndef FX_Q8_WAVES
#define FX_Q8_WAVES 1  // minimum waves per SIMD for the quint8 kernels (4: <= 128 VGPRs)
#endif
template <typename T>
constexpr int kMinWaves = sizeof(T) == 1 ? FX_Q8_WAVES : 1;

template <typename T, int W, int L, int U, int METRIC, bool PIPE, bool DMA = false>
__global__ void __launch_bounds__(256, kMinWaves<T>) scan_kernel(ScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int S = a.d / W;
  constexpr int CH = 16 * L;
  const int nch = (S + CH - 1) / CH;
  const int qfl = nch * CH * W;  // padded query floats

  float* q_lds = reinterpret_cast<float*>(smem);
  const int qi = blockIdx.y;
  // the batched path's overflow fallback: only queries whose count overflowed
  if (a.gate != nullptr && (int64_t)a.gate[(size_t)qi * kCountStride] <= a.gate_cap) return;
  const float* qg = a.q + (size_t)qi * a.d;
  for (int i = threadIdx.x; i < qfl; i += 256) {
    float v = i < a.d ? qg[i] : 0.f;
    // quint8 L2: q' = qshift + q / qscale (padding -> qshift, which the padded
    // zero-point codes cancel exactly)
    if constexpr (sizeof(T) == 1 && METRIC == 0) v = a.qshift + v / a.qscale;
    q_lds[i] = v;
  }
  __syncthreads();

  ScanCtx c;
  c.a = &a;
  c.q_lds = q_lds;
  c.buf = reinterpret_cast<uint64_t*>(smem + a.qbytes) + (size_t)wid * a.cap;
  c.hist = reinterpret_cast<uint32_t*>(smem + a.qbytes + (size_t)4 * a.cap * 8) + wid * 256;
  c.S = S;
  c.lane = lane;
  c.grp = lane >> 4;
  c.jl = lane & 15;
  c.qi = qi;
  c.qnorm = 1.f;
  c.qscale = a.qscale;
  c.qshift = a.qshift;
  c.topk = a.mode == kModeTopk;
  if constexpr (METRIC == 2) {
    // F.normalize eps (coder.py:43-44): max(||q||, 1e-12); every wave reduces
    // the LDS copy itself so no extra barrier is needed.
    float s2 = 0.f;
    for (int i = lane; i < a.d; i += kWave) s2 = fmaf(q_lds[i], q_lds[i], s2);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s2 += __shfl_xor(s2, m);
    c.qnorm = fmaxf(sqrtf(s2), 1e-12f);
  }

  // A block step is 16U rows (4U per wave).  Contiguous: block b owns one
  // range of rows_per_block.  Interleaved: block steps are dealt round-robin
  // over the grid, so at any time the whole chip reads one window of the
  // corpus (DRAM pages stay open across CUs: tools/hbm_sweep.hip).  Either
  // partition gives the same result (the merge orders by (distance, row)).
  const int64_t step = 16 * U;
  int64_t lo, gstep;
  if (a.interleave & 1) {
    lo = (int64_t)blockIdx.x * step;
    c.hi = a.n;
    gstep = (int64_t)gridDim.x * step;
  } else {
    lo = (int64_t)blockIdx.x * a.rows_per_block;
    c.hi = lo + a.rows_per_block < a.n ? lo + a.rows_per_block : a.n;
    gstep = step;
  }

  uint64_t thr = kEmpty;
  int cnt = 0;
  RowTile<T, W, L, U> tA, tB;

  if constexpr (DMA) {
    // Per-wave ring of FX_Q8DMA_STAGES tiles after the block's LDS: one
    // global_load_lds per 16-B slot column (64 lanes x 16 B = the wave's 4U
    // rows' slot cc), issued FX_Q8DMA_STAGES - 1 tiles ahead; the counted
    // vmcnt leaves the later tiles in flight.  Slots past the row end read a
    // valid dummy and are replaced by the zero-point code in registers; rows
    // past the range are clamped to its last row (never consumed).  One pass
    // per row (nch == 1), no mask, no row list (plan_scan / launch_scan).
    constexpr int R = FX_Q8DMA_STAGES;
    constexpr int kTileBytes = U * L * 1024;
    unsigned char* ring = smem + a.qbytes + (size_t)4 * a.cap * 8 + 4 * 256 * 4 +
                          (size_t)__builtin_amdgcn_readfirstlane(wid) * R * kTileBytes;
    const int64_t first = lo + (int64_t)wid * 4 * U;
    const int64_t ntile = first < c.hi ? (c.hi - first + gstep - 1) / gstep : 0;
    using V = typename VecT<T, W>::type;
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef float f16v __attribute__((ext_vector_type(16)));
    static_assert(W == 16, "the DMA path scans 16 quint8 codes per lane slot");
    const f2 z2 = {c.qshift, c.qshift};
    f2 qreg[L][8];  // this lane's query slots (jl, jl + 16, ...), held in registers
#pragma unroll
    for (int cc = 0; cc < L; ++cc) {
      const f2* qp = reinterpret_cast<const f2*>(c.q_lds + (cc * 16 + c.jl) * W);
#pragma unroll
      for (int p = 0; p < 8; ++p) qreg[cc][p] = qp[p];
    }
    int slot_i = 0, slot_n = R - 1;
#pragma unroll
    for (int j = 0; j < R - 1; ++j) {
        const int64_t jj = j;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          int64_t row = first + jj * gstep + u * 4 + c.grp;
          if (row >= c.hi) row = c.hi - 1;
#pragma unroll
          for (int cc = 0; cc < L; ++cc) {
            const int sl = cc * 16 + c.jl;
            const void* g = reinterpret_cast<const T*>(a.X) + row * (int64_t)a.d + (sl < S ? sl : 0) * 16;
            __builtin_amdgcn_global_load_lds(
                g, (__attribute__((address_space(3))) void*)(ring + j * kTileBytes + (u * L + cc) * 1024),
                16, 0, FX_Q8DMA_AUX);
          }
        }
      }
    for (int64_t i = 0; i < ntile; ++i) {
      {
        const int64_t jj = i + R - 1;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          int64_t row = first + jj * gstep + u * 4 + c.grp;
          if (row >= c.hi) row = c.hi - 1;
#pragma unroll
          for (int cc = 0; cc < L; ++cc) {
            const int sl = cc * 16 + c.jl;
            const void* g = reinterpret_cast<const T*>(a.X) + row * (int64_t)a.d + (sl < S ? sl : 0) * 16;
            __builtin_amdgcn_global_load_lds(
                g, (__attribute__((address_space(3))) void*)(ring + slot_n * kTileBytes + (u * L + cc) * 1024),
                16, 0, FX_Q8DMA_AUX);
          }
        }
      }
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((R - 1) * U * L) : "memory");
      RowTile<T, W, L, U> t;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        t.row[u] = first + i * gstep + u * 4 + c.grp;
        t.valid[u] = t.row[u] < c.hi;
        t.src[u] = t.row[u];
#pragma unroll
        for (int cc = 0; cc < L; ++cc) {
          t.v[u][cc] = *reinterpret_cast<const V*>(ring + slot_i * kTileBytes +
                                                   (u * L + cc) * 1024 + lane * 16);
          if (cc * 16 + c.jl >= S) t.v[u][cc] = V((T)c.qshift);  // dequantises to 0
        }
      }
      // tile_accumulate's quint8 arithmetic, operation for operation (so the
      // distances equal the register-tile path's), with the query in registers
      float acc[U], acc2[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc[u] = acc2[u] = 0.f;
#pragma unroll
        for (int cc = 0; cc < L; ++cc) {
          const f16v xf = __builtin_convertvector(t.v[u][cc], f16v);
          f2 a2 = {0.f, 0.f}, b2 = {0.f, 0.f};
#pragma unroll
          for (int p = 0; p < 8; ++p) {
            const f2 x2 = {xf[2 * p], xf[2 * p + 1]};
            if constexpr (METRIC == 0) {
              const f2 dd = x2 - qreg[cc][p];
              a2 = __builtin_elementwise_fma(dd, dd, a2);
            } else {
              const f2 dd = x2 - z2;
              a2 = __builtin_elementwise_fma(dd, qreg[cc][p], a2);
              if constexpr (METRIC == 2) b2 = __builtin_elementwise_fma(dd, dd, b2);
            }
          }
          acc[u] += a2.x + a2.y;
          if constexpr (METRIC == 2) acc2[u] += b2.x + b2.y;
        }
      }
      tile_finish<T, W, L, U, METRIC>(t, acc, acc2, c, thr, cnt);
      slot_i = slot_i == R - 1 ? 0 : slot_i + 1;
      slot_n = slot_n == R - 1 ? 0 : slot_n + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's tail loads
  } else if (PIPE && nch == 1 && !(a.interleave & 2)) {
    int64_t it = lo + (int64_t)wid * 4 * U;
    if (it < c.hi) tile_load(tA, it, 0, c);
    for (; it < c.hi; it += 2 * gstep) {
      const int64_t it1 = it + gstep;
      if (it1 < c.hi) tile_load(tB, it1, 0, c);
      tile_consume<T, W, L, U, METRIC>(tA, c, thr, cnt);
      if (it1 >= c.hi) break;
      const int64_t it2 = it1 + gstep;
      if (it2 < c.hi) tile_load(tA, it2, 0, c);
      tile_consume<T, W, L, U, METRIC>(tB, c, thr, cnt);
    }
  } else {
    // rows longer than one pass (d > 16*L*W): accumulate pass by pass
    for (int64_t it = lo + (int64_t)wid * 4 * U; it < c.hi; it += gstep) {
      float acc[U], acc2[U];
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = acc2[u] = 0.f;
      for (int ch = 0; ch < nch; ++ch) {
        tile_load(tA, it, ch, c);
        tile_accumulate<T, W, L, U, METRIC>(tA, ch, c, acc, acc2);
      }
      tile_finish<T, W, L, U, METRIC>(tA, acc, acc2, c, thr, cnt);
    }
  }

  if (!c.topk) return;
  wave_sync();
  if (cnt > a.k) {
    int quota;
    const uint64_t kth = wave_select(c.buf, cnt, a.k, c.hist, lane, &quota);
    cnt = wave_compact(c.buf, cnt, kth, quota, lane);
  }
  // Fold the block's 4 wave lists (k each, padded) into one list of k:
  // a quarter of the candidates for the merge kernels (block-wide select).
  constexpr int kMaxPerLane = 16;  // k <= 1024
  uint64_t mine[kMaxPerLane];
#pragma unroll
  for (int j = 0; j < kMaxPerLane; ++j) {
    const int i = lane + j * kWave;
    mine[j] = i < cnt ? c.buf[i] : kEmpty;
  }
  __syncthreads();
  uint64_t* all = reinterpret_cast<uint64_t*>(smem + a.qbytes);  // 4k entries fit in 4 caps
  uint64_t v_or = 0, v_and = ~0ull;
#pragma unroll
  for (int j = 0; j < kMaxPerLane; ++j) {
    const int i = lane + j * kWave;
    if (i < a.k) {
      all[wid * a.k + i] = mine[j];
      v_or |= mine[j];
      v_and &= mine[j];
    }
  }
  MergeShared* ms = reinterpret_cast<MergeShared*>(smem + a.qbytes + (size_t)4 * a.cap * 8);
  block_reset(ms);
  __syncthreads();
  block_or_and(v_or, v_and, ms);
  __syncthreads();
  const size_t ls = a.list_stride > 0 ? (size_t)a.list_stride : (size_t)gridDim.x;
  uint64_t* out = a.out_lists + ((size_t)qi * ls + a.list_base + blockIdx.x) * (size_t)a.k;
  block_keep_k<256>(all, 4 * a.k, a.k, out, ms);
}

// ----------------------------------------------------- dispatch / planning --

#ifndef FX_SCAN_INTERLEAVE_DEFAULT
#define FX_SCAN_INTERLEAVE_DEFAULT 1
#endif
static constexpr int kInterleaveDefault = FX_SCAN_INTERLEAVE_DEFAULT;

// Double-buffered tiles everywhere except 16-bit rows of >= 12 slots, where
// the second tile (plus the f16->f32 converts) costs more occupancy than the
// overlap gains (tools/microbench.py sweep, profiles/r01_microbench_*.log).
template <typename T, int L>
constexpr bool kPipe = !(sizeof(T) == 2 && L >= 12);

template <typename T, int W, int METRIC>
static ScanKernelFn pick_l(int L) {
  if constexpr (sizeof(T) == 1) {
    switch (L) {
      case 1: return scan_kernel<T, W, 1, FX_Q1, METRIC, true>;
      case 2: return scan_kernel<T, W, 2, FX_Q2, METRIC, true>;
      case 3: return scan_kernel<T, W, 3, FX_Q3, METRIC, true>;
      case 4: return scan_kernel<T, W, 4, FX_Q4, METRIC, true>;
      case 6: return scan_kernel<T, W, 6, FX_Q6, METRIC, true>;
      case 8: return scan_kernel<T, W, 8, FX_Q8, METRIC, true>;
      case 12: return scan_kernel<T, W, 12, FX_Q12, METRIC, true>;
      case 16: return scan_kernel<T, W, 16, 1, METRIC, true>;
      default: return scan_kernel<T, W, 24, 1, METRIC, true>;
    }
  } else {
    switch (L) {
      case 1: return scan_kernel<T, W, 1, FX_U1, METRIC, kPipe<T, 1>>;
      case 2: return scan_kernel<T, W, 2, FX_U2, METRIC, kPipe<T, 2>>;
      case 3: return scan_kernel<T, W, 3, FX_U3, METRIC, kPipe<T, 3>>;
      case 4: return scan_kernel<T, W, 4, FX_U4, METRIC, kPipe<T, 4>>;
      case 6: return scan_kernel<T, W, 6, FX_U6, METRIC, kPipe<T, 6>>;
      case 8: return scan_kernel<T, W, 8, FX_U8, METRIC, kPipe<T, 8>>;
      case 12: return scan_kernel<T, W, 12, FX_U12, METRIC, kPipe<T, 12>>;
      case 16: return scan_kernel<T, W, 16, 1, METRIC, kPipe<T, 16>>;
      default: return scan_kernel<T, W, 24, 1, METRIC, kPipe<T, 24>>;
    }
  }
}

template <typename T, int METRIC>
static ScanKernelFn pick_scalar() {
  return scan_kernel<T, 1, 16, 1, METRIC, true>;
}

static int rows_unroll_q8(int L) {
  switch (L) {
    case 1: return FX_Q1;
    case 2: return FX_Q2;
    case 3: return FX_Q3;
    case 4: return FX_Q4;
    case 6: return FX_Q6;
    case 8: return FX_Q8;
    case 12: return FX_Q12;
    default: return 1;
  }
}

static int rows_unroll(int L) {
  switch (L) {
    case 1: return FX_U1;
    case 2: return FX_U2;
    case 3: return FX_U3;
    case 4: return FX_U4;
    case 6: return FX_U6;
    case 8: return FX_U8;
    case 12: return FX_U12;
    default: return 1;
  }
}

template <int METRIC>
static ScanKernelFn pick_q8_dma(int L) {
  constexpr int U = FX_Q8DMA_U;
  switch (L) {
    case 1: return scan_kernel<uint8_t, 16, 1, U, METRIC, true, true>;
    case 2: return scan_kernel<uint8_t, 16, 2, U, METRIC, true, true>;
    case 3: return scan_kernel<uint8_t, 16, 3, U, METRIC, true, true>;
    case 4: return scan_kernel<uint8_t, 16, 4, U, METRIC, true, true>;
    default: return nullptr;
  }
}

static ScanKernelFn select_q8_dma_kernel(int metric, int L) {
  if (metric == 0) return pick_q8_dma<0>(L);
  if (metric == 1) return pick_q8_dma<1>(L);
  return pick_q8_dma<2>(L);
}

ScanKernelFn select_scan_kernel(int dtype, int metric, int W, int L) {
  if (dtype == FX_DTYPE_F32) {
    if (W == 1) {
      if (metric == 0) return pick_scalar<float, 0>();
      if (metric == 1) return pick_scalar<float, 1>();
      return pick_scalar<float, 2>();
    }
    if (metric == 0) return pick_l<float, 4, 0>(L);
    if (metric == 1) return pick_l<float, 4, 1>(L);
    return pick_l<float, 4, 2>(L);
  }
  if (dtype == FX_DTYPE_QU8) {
    if (W == 1) {
      if (metric == 0) return pick_scalar<uint8_t, 0>();
      if (metric == 1) return pick_scalar<uint8_t, 1>();
      return pick_scalar<uint8_t, 2>();
    }
    if (metric == 0) return pick_l<uint8_t, 16, 0>(L);
    if (metric == 1) return pick_l<uint8_t, 16, 1>(L);
    return pick_l<uint8_t, 16, 2>(L);
  }
  if (W == 1) {
    if (metric == 0) return pick_scalar<_Float16, 0>();
    if (metric == 1) return pick_scalar<_Float16, 1>();
    return pick_scalar<_Float16, 2>();
  }
  if (metric == 0) return pick_l<_Float16, 8, 0>(L);
  if (metric == 1) return pick_l<_Float16, 8, 1>(L);
  return pick_l<_Float16, 8, 2>(L);
}

// Shape → kernel variant, LDS size, grid.  Pure function of (shape, device).
int plan_scan(int64_t n, int64_t d, int dtype, int64_t k, int metric, bool aligned,
              ScanPlan* p) {
  const int vecw = dtype == FX_DTYPE_F32 ? 4 : dtype == FX_DTYPE_F16 ? 8 : 16;
  int W = (aligned && d % vecw == 0) ? vecw : 1;
  const int64_t S = d / W;
  int L;
  if (W == 1) {
    L = 16;
  } else {
    const int64_t need = (S + 15) / 16;
    static const int choices[] = {1, 2, 3, 4, 6, 8, 12, 16, 24};
    L = 24;
    for (int c : choices) {
      if (c >= need) {
        L = c;
        break;
      }
    }
  }
  const int U = W == 1 ? 1 : dtype == FX_DTYPE_QU8 ? rows_unroll_q8(L) : rows_unroll(L);
  const int64_t CH = 16 * (int64_t)L;
  const int64_t nch = (S + CH - 1) / CH;
  const size_t qbytes = (size_t)((nch * CH * W * 4 + 15) / 16 * 16);
  int cap = 256;
  while (cap < 2 * k || cap - 4 * U < k) cap *= 2;
  const size_t smem = qbytes + (size_t)4 * cap * 8 + (size_t)4 * 256 * 4;
  if (smem > 160 * 1024) {
    set_error("k=%lld with d=%lld needs %zu bytes of LDS per workgroup (max 163840)",
              (long long)k, (long long)d, smem);
    return FX_EUNSUPPORTED;
  }
  p->fn = select_scan_kernel(dtype, metric, W, L);
  p->fn_dma = nullptr;
  p->smem_dma = 0;
  if (dtype == FX_DTYPE_QU8 && W == 16 && nch == 1 && U % FX_Q8DMA_U == 0) {
    const size_t sd = smem + (size_t)4 * FX_Q8DMA_STAGES * FX_Q8DMA_U * L * 1024;
    if (sd <= 80 * 1024 && option(kOptQ8Dma) != 0) {  // >= 2 workgroups per CU
      p->fn_dma = select_q8_dma_kernel(metric, L);
      p->smem_dma = sd;
    }
  }
  p->W = W;
  p->L = L;
  p->U = U;
  p->cap = cap;
  p->qbytes = qbytes;
  p->smem = smem;
  int cus = 0, occ = 0;
  int rc = device_cus(&cus);
  if (rc) return rc;
  rc = kernel_occupancy((const void*)p->fn, 256, smem, &occ);
  if (rc) return rc;
  if (p->fn_dma != nullptr) {  // one grid serves both variants: the smaller occupancy
    int occ2 = 0;
    // the DMA variants may take more than the default 64 KB of dynamic LDS
    rc = allow_lds((const void*)p->fn_dma);
    if (rc) return rc;
    rc = kernel_occupancy((const void*)p->fn_dma, 256, p->smem_dma, &occ2);
    if (rc) return rc;
    if (occ2 < occ) occ = occ2;
  }
  // Two 256-thread blocks per CU already saturate HBM with the pipelined
  // tiles (sweep in profiles/), and fewer blocks mean fewer candidate lists
  // to merge.  FX_SCAN_BLOCKS_PER_CU overrides (diagnostic builds, microbench).
  // Rows of >= 12 slots per lane (768-d f32, 1536-d f16 and longer): one
  // block per CU reads as fast or faster (1536-d f16: 4.50 vs 4.66 ms).
  const int cap_occ =
      diag_env("FX_SCAN_BLOCKS_PER_CU", dtype == FX_DTYPE_QU8 ? 3 : L >= 12 ? 1 : 2);
  if (cap_occ > 0 && cap_occ < occ) occ = cap_occ;
  if (occ < 1) occ = 1;
  const int64_t max_blocks = (int64_t)cus * occ;
  // at least 2 k rows per block (k / 2 per wave): fewer rows than that and
  // the lists outweigh the rows; more (8 k, before round 4) left most CUs
  // idle on small shards at large k -- 500k x 1536 fp16, k = 1000: 62 blocks,
  // 0.78 ms; 245 blocks, 0.33 ms (6.25M rows and k = 100 unchanged,
  // profiles/r04_scan_min_rows.jsonl)
#ifndef FX_SCAN_MIN_ROWS_K
#define FX_SCAN_MIN_ROWS_K 2
#endif
  int64_t min_rows = 16 * U * 4;
  if (min_rows < FX_SCAN_MIN_ROWS_K * k) min_rows = FX_SCAN_MIN_ROWS_K * k;
  if (min_rows < 256) min_rows = 256;
  int64_t blocks = (n + min_rows - 1) / min_rows;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks < 1) blocks = 1;
  int64_t rpb = (n + blocks - 1) / blocks;
  const int64_t step = 16 * U;
  rpb = (rpb + step - 1) / step * step;
  blocks = (n + rpb - 1) / rpb;
  if (blocks < 1) blocks = 1;
  p->blocks = blocks;
  p->rows_per_block = rpb > 0 ? rpb : step;
  p->nlists = blocks;  // one list per block (the epilogue folds its 4 waves)
  // Block steps dealt round-robin over the grid for rows of >= 1 KB, each
  // block one contiguous range below that (sweep over d and dtype:
  // profiles/r02_scan_interleave_sweep.log).  The "scan_interleave" option
  // (test switch) overrides.
  const int esize = dtype == FX_DTYPE_F32 ? 4 : dtype == FX_DTYPE_F16 ? 2 : 1;
  p->interleave = kInterleaveDefault && d * esize >= 1024;
  if (option(kOptScanInterleave) >= 0) p->interleave = option(kOptScanInterleave) != 0;
  // FX_SCAN_PIPE=0: one register tile per wave in flight (diagnostic builds)
  if (diag_env("FX_SCAN_PIPE", 1) == 0) p->interleave |= 2;
  return FX_OK;
}

void limit_scan_blocks(ScanPlan* p, int64_t n, int64_t max_blocks) {
  if (max_blocks < 1 || p->blocks <= max_blocks) return;
  const int64_t step = 16 * (int64_t)p->U;
  int64_t rpb = (n + max_blocks - 1) / max_blocks;
  rpb = (rpb + step - 1) / step * step;
  p->rows_per_block = rpb > 0 ? rpb : step;
  p->blocks = (n + p->rows_per_block - 1) / p->rows_per_block;
  if (p->blocks < 1) p->blocks = 1;
  p->nlists = p->blocks;
}

int launch_scan(const ScanPlan& p, const ScanArgs& a, int64_t nq, hipStream_t stream) {
  dim3 grid((unsigned)p.blocks, (unsigned)nq);
  if (p.fn_dma != nullptr && a.mask == nullptr && a.rows == nullptr) {
    if (int rc = allow_lds((const void*)p.fn_dma)) return rc;
    ScanArgs b = a;
    b.interleave = p.interleave & 1;
    hipLaunchKernelGGL(p.fn_dma, grid, dim3(256), p.smem_dma, stream, b);
    return check_launch("scan_kernel (quint8 LDS-DMA)");
  }
  if (p.smem > 64 * 1024) {
    if (int rc = allow_lds((const void*)p.fn)) return rc;
  }
  ScanArgs b = a;
  b.interleave = p.interleave;
  hipLaunchKernelGGL(p.fn, grid, dim3(256), p.smem, stream, b);
  return check_launch("scan_kernel");
}

}  // namespace fx
