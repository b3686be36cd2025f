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
#include "fx_internal.h"
#include "fx_wave.h"

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
  for (int shift = 56; shift >= 0; shift -= 8) {
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
// passes if the row is longer); U: rows per lane group in flight.

template <typename T, int W, int L, int U, int METRIC>
__global__ void __launch_bounds__(256) scan_kernel(ScanArgs a) {
  using V = typename VecT<T, W>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int grp = lane >> 4, jl = lane & 15;
  const int S = a.d / W;
  constexpr int CH = 16 * L;
  const int nch = (S + CH - 1) / CH;
  const int qfl = nch * CH * W;  // padded query floats

  float* q_lds = reinterpret_cast<float*>(smem);
  uint64_t* buf = reinterpret_cast<uint64_t*>(smem + a.qbytes) + (size_t)wid * a.cap;
  uint32_t* hist =
      reinterpret_cast<uint32_t*>(smem + a.qbytes + (size_t)4 * a.cap * 8) + wid * 256;

  const int qi = blockIdx.y;
  const float* qg = a.q + (size_t)qi * a.d;
  for (int i = threadIdx.x; i < qfl; i += 256) q_lds[i] = i < a.d ? qg[i] : 0.f;
  __syncthreads();
  float qnorm = 1.f;
  if constexpr (METRIC == 2) {
    // F.normalize eps (coder.py:43-44): max(||q||, 1e-12); every wave reduces
    // the LDS copy itself so no extra barrier is needed.
    float s2 = 0.f;
    for (int i = lane; i < a.d; i += kWave) s2 = fmaf(q_lds[i], q_lds[i], s2);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s2 += __shfl_xor(s2, m);
    qnorm = fmaxf(sqrtf(s2), 1e-12f);
  }

  const T* X = reinterpret_cast<const T*>(a.X);
  const int64_t lo = (int64_t)blockIdx.x * a.rows_per_block;
  const int64_t hi = lo + a.rows_per_block < a.n ? lo + a.rows_per_block : a.n;
  const bool topk = a.mode == kModeTopk;

  uint64_t thr = kEmpty;
  int cnt = 0;

  for (int64_t it = lo + (int64_t)wid * 4 * U; it < hi; it += 16 * U) {
    int64_t row[U];
    bool valid[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      row[u] = it + u * 4 + grp;
      valid[u] = row[u] < hi;
      if (a.mask != nullptr && valid[u]) valid[u] = (a.mask[row[u] >> 5] >> (row[u] & 31)) & 1u;
    }
    float acc[U], acc2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = acc2[u] = 0.f;

    for (int ch = 0; ch < nch; ++ch) {
      V v[U][L];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const V* rp = reinterpret_cast<const V*>(X + row[u] * (int64_t)a.d);
#pragma unroll
        for (int c = 0; c < L; ++c) {
          const int s = ch * CH + c * 16 + jl;
          if (valid[u] && s < S) {
            v[u][c] = load_stream(rp + s);
          } else {
            v[u][c] = V(0);
          }
        }
      }
#pragma unroll
      for (int c = 0; c < L; ++c) {
        const int s = ch * CH + c * 16 + jl;
        float qv[W];
#pragma unroll
        for (int e = 0; e < W; ++e) qv[e] = q_lds[s * W + e];
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int e = 0; e < W; ++e) {
            const float x = elem<W>(v[u][c], e);
            if constexpr (METRIC == 0) {
              const float t = x - qv[e];
              acc[u] = fmaf(t, t, acc[u]);
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

    float dist[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float s1 = sum16(acc[u]);
      if constexpr (METRIC == 0) {
        dist[u] = sqrtf(s1);
      } else if constexpr (METRIC == 1) {
        dist[u] = -s1;
      } else {
        const float s2 = sum16(acc2[u]);
        const float nx = fmaxf(sqrtf(s2), 1e-12f);
        dist[u] = 0.5f - 0.5f * (s1 / (nx * qnorm));
      }
    }

    if (!topk) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (jl == 0 && row[u] < hi)
          a.out_dist[(size_t)qi * a.n + row[u]] = valid[u] ? dist[u] : __builtin_nanf("");
      }
      continue;
    }

    const uint64_t ltmask = (1ull << lane) - 1ull;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t comp = make_comp(dist[u], (uint32_t)(a.row_base + row[u]));
      const bool p = (jl == 0) && valid[u] && comp < thr;
      const uint64_t b = __ballot(p);
      if (b) {
        if (p) buf[cnt + __popcll(b & ltmask)] = comp;
        cnt += __popcll(b);
      }
    }
    if (cnt > a.cap - 4 * U) {
      wave_sync();
      int quota;
      thr = wave_select(buf, cnt, a.k, hist, lane, &quota);
      cnt = wave_compact(buf, cnt, thr, quota, lane);
    }
  }

  if (!topk) return;
  wave_sync();
  if (cnt > a.k) {
    int quota;
    const uint64_t kth = wave_select(buf, cnt, a.k, hist, lane, &quota);
    cnt = wave_compact(buf, cnt, kth, quota, lane);
  }
  uint64_t* out =
      a.out_lists + ((size_t)qi * gridDim.x * 4 + (size_t)blockIdx.x * 4 + wid) * (size_t)a.k;
  for (int i = lane; i < a.k; i += kWave) out[i] = i < cnt ? buf[i] : kEmpty;
}

// ----------------------------------------------------- dispatch / planning --

template <typename T, int W, int METRIC>
static ScanKernelFn pick_l(int L) {
  switch (L) {
    case 1: return scan_kernel<T, W, 1, 8, METRIC>;
    case 2: return scan_kernel<T, W, 2, 4, METRIC>;
    case 3: return scan_kernel<T, W, 3, 2, METRIC>;
    case 4: return scan_kernel<T, W, 4, 2, METRIC>;
    case 6: return scan_kernel<T, W, 6, 1, METRIC>;
    case 8: return scan_kernel<T, W, 8, 1, METRIC>;
    case 12: return scan_kernel<T, W, 12, 1, METRIC>;
    case 16: return scan_kernel<T, W, 16, 1, METRIC>;
    default: return scan_kernel<T, W, 24, 1, METRIC>;
  }
}

template <typename T, int METRIC>
static ScanKernelFn pick_scalar() {
  return scan_kernel<T, 1, 16, 1, METRIC>;
}

static int rows_unroll(int L) {
  switch (L) {
    case 1: return 8;
    case 2: return 4;
    case 3: return 2;
    case 4: return 2;
    default: return 1;
  }
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
  const int vecw = dtype == FX_DTYPE_F32 ? 4 : 8;
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
  const int U = W == 1 ? 1 : rows_unroll(L);
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
  if (occ < 1) occ = 1;
  const int64_t max_blocks = (int64_t)cus * occ;
  // each wave should see many more rows than k for the threshold to filter
  int64_t min_rows = 16 * U * 4;
  if (min_rows < 8 * k) min_rows = 8 * k;
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
  p->nlists = blocks * 4;
  return FX_OK;
}

int launch_scan(const ScanPlan& p, const ScanArgs& a, int64_t nq, hipStream_t stream) {
  dim3 grid((unsigned)p.blocks, (unsigned)nq);
  hipLaunchKernelGGL(p.fn, grid, dim3(256), p.smem, stream, a);
  return check_launch("scan_kernel");
}

}  // namespace fx
