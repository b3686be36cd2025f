// Merge of per-wave / per-shard candidate lists into the final sorted top-k.
//
// Replaces the global select of the reference: pc.select_k_unstable over the
// whole (multi-source concatenated) table, src/fenix/io/index/index.py:165-168
// (sources concatenated by src/fenix/io/table/table.py:19-21,35).
//
// Each level: one 256-thread workgroup loads G lists (<= kMergeEntries
// composites) into LDS, finds the k-th composite with a block-wide 8-bit
// radix select, and keeps the k smallest.  Levels repeat until one list per
// query remains; the last level bitonic-sorts it and decodes composites back
// to (distance f32, row i64).  The candidate SET is deterministic at every
// level (composites are unique), so the sorted output is bit-reproducible.
// Workgroups are 1024 threads: a 256-thread group left each level latency-
// bound (~40 us per 8 K entries, 140 us for the k = 1000 final level).
#include <stdlib.h>

#include "fx_internal.h"
#include "fx_select.h"

namespace fx {

constexpr int kMergeThreads = 1024;  // 16 waves: latency hiding for the LDS passes
// 128 KB of composites per workgroup: the batched path's 16 K-entry candidate
// buffers (4 lists of 4 096) fold in one level (one launch, 16-20 us less
// per threshold than two levels of 8 K)
#ifndef FX_MERGE_ENTRIES
#define FX_MERGE_ENTRIES 16384
#endif
constexpr int64_t kMergeEntries = FX_MERGE_ENTRIES;

__global__ void __launch_bounds__(kMergeThreads)
    merge_kernel(const uint64_t* __restrict__ in, int64_t nlists, int kin, int64_t G, int k,
                 int P2, uint64_t* __restrict__ out_lists, float* __restrict__ out_dist,
                 int64_t* __restrict__ out_row, uint64_t* __restrict__ out_kth,
                 int final_level, const uint32_t* __restrict__ gate, int64_t gate_cap,
                 uint32_t* __restrict__ count, int zero_count) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  MergeShared* ms = reinterpret_cast<MergeShared*>(smem);
  uint64_t* res = reinterpret_cast<uint64_t*>(smem + sizeof(MergeShared));
  const int rcap = P2 > k ? P2 : k;
  uint64_t* s = res + rcap;

  const int tid = threadIdx.x;
  const int q = blockIdx.y;
  // the batched path's overflow fallback merges only the recomputed queries
  if (gate != nullptr && (int64_t)gate[(size_t)q * kCountStride] <= gate_cap) return;
  const int64_t l0 = (int64_t)blockIdx.x * G;
  const int nl = (int)((nlists - l0) < G ? (nlists - l0) : G);
  int m = nl * kin;
  if (count != nullptr) {  // appended lists: only the first count[q] slots hold entries
    const int64_t c = (int64_t)count[(size_t)q * kCountStride];
    const int64_t all = nlists * kin;
    const int64_t valid = (c < all ? c : all) - l0 * kin;
    m = valid < 0 ? 0 : (valid < m ? (int)valid : m);
  }
  const uint64_t* src = in + ((size_t)q * nlists + l0) * (size_t)kin;
  block_reset(ms);
  __syncthreads();
  // (every thread has read count: the next phase's appends may start from 0)
  if (zero_count && tid == 0) count[(size_t)q * kCountStride] = 0u;
  uint64_t v_or = 0, v_and = ~0ull;
  // 8 loads in flight per thread: one dependent load per iteration made every
  // level latency-bound (~50 us for 8 K entries).
  for (int base = tid; base < m; base += kMergeThreads * 8) {
    uint64_t e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = base + j * kMergeThreads;
      e[j] = i < m ? src[i] : kEmpty;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = base + j * kMergeThreads;
      if (i < m) {
        s[i] = e[j];
        v_or |= e[j];
        v_and &= e[j];
      }
    }
  }
  block_or_and(v_or, v_and, ms);
  __syncthreads();

  // a threshold only (the batched filter's sampling phases): the k-th
  // smallest composite is the select's threshold, no keep / sort needed
  if (final_level && out_kth != nullptr && out_dist == nullptr && gridDim.x == 1) {
    uint64_t kth = kEmpty;  // fewer than k entries: no threshold
    if (m > k) {
      const uint64_t diff = ms->all_or ^ ms->all_and;
      const int start_shift = diff ? (63 - __clzll((long long)diff)) / 8 * 8 : 0;
      int quota;
      kth = block_select<kMergeThreads>(s, m, k, start_shift, ms->all_and, ms, &quota);
    } else if (m == k) {  // exactly k entries: the k-th smallest is the largest
      uint64_t mx = 0ull;
      for (int i = tid; i < m; i += kMergeThreads) mx = s[i] > mx ? s[i] : mx;
      mx = wave_max_u64(mx);
      if (tid == 0) ms->shmax = 0ull;
      __syncthreads();
      if ((tid & 63) == 0) atomicMax(&ms->shmax, (unsigned long long)mx);
      __syncthreads();
      kth = ms->shmax;
    }
    if (tid == 0 && kth < out_kth[q]) out_kth[q] = kth;
    return;
  }

  int nres;
  if (m > k) {
    block_keep_k<kMergeThreads>(s, m, k, res, ms);
    nres = k;
  } else {
    for (int i = tid; i < m; i += kMergeThreads) res[i] = s[i];
    nres = m;
  }
  __syncthreads();
  const int fill_to = final_level ? P2 : k;
  for (int i = nres + tid; i < fill_to; i += kMergeThreads) res[i] = kEmpty;
  __syncthreads();

  if (!final_level) {
    uint64_t* dst = out_lists + ((size_t)q * gridDim.x + blockIdx.x) * (size_t)k;
    for (int i = tid; i < k; i += kMergeThreads) dst[i] = res[i];
    return;
  }

  // bitonic sort of res[0..P2): one compare-swap per thread per stage
  for (int size = 2; size <= P2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < (P2 >> 1); i += kMergeThreads) {
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
  uint64_t* sorted = res;
  res = sorted;
  // (a threshold only tightens: a phase with fewer than k candidates, or
  // whose k-th is above the previous one, keeps the previous)
  if (out_kth != nullptr && tid == 0 && res[k - 1] < out_kth[q]) out_kth[q] = res[k - 1];
  if (out_dist == nullptr) return;
  for (int i = tid; i < k; i += kMergeThreads) {
    const uint64_t e = res[i];
    float dv;
    int64_t rv;
    if (e == kEmpty) {
      dv = __builtin_nanf("");
      rv = -1;
    } else {
      dv = key_float((uint32_t)(e >> 32));
      rv = (int64_t)(e & 0xffffffffull);
    }
    out_dist[(size_t)q * k + i] = dv;
    out_row[(size_t)q * k + i] = rv;
  }
}

static int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

int plan_merge(int64_t nq, int64_t nlists, int64_t kin, int64_t k, MergePlan* p) {
  if (kin > kMergeEntries / 2 || k > kMergeEntries / 2) {
    set_error("merge list length %lld / k %lld exceeds %lld", (long long)kin, (long long)k,
              (long long)(kMergeEntries / 2));
    return FX_EUNSUPPORTED;
  }
  p->levels = 0;
  int64_t lists = nlists, klen = kin;
  size_t scratch = 0;
  while (true) {
    if (p->levels >= 16) {
      set_error("merge tree too deep");
      return FX_EUNSUPPORTED;
    }
    // >= 3.2 K entries per 1024-thread workgroup: few levels, each still
    // spread over many CUs (tools/microbench.py reduce[group=*]).
    const int64_t target = 8 * klen > 3200 ? 8 * klen : 3200;
    int64_t G = (target + klen - 1) / klen;
    if (G * klen > kMergeEntries) G = kMergeEntries / klen;
    {  // FX_MERGE_GROUP: tuning knob of diagnostic builds (tools/microbench.py)
      const int64_t g = diag_env("FX_MERGE_GROUP", 0);
      if (g >= 2 && g * klen <= kMergeEntries) G = g;
    }
    if (G < 2) G = 2;
    if (G > lists) G = lists;
    const int64_t next = (lists + G - 1) / G;
    p->group[p->levels] = G;
    p->lists[p->levels] = lists;
    p->klen[p->levels] = klen;
    p->levels++;
    if (next > 1) {
      const size_t bytes = (size_t)nq * next * k * 8;
      if (bytes > scratch) scratch = bytes;
    }
    lists = next;
    klen = k;
    if (lists == 1) break;
  }
  p->lists[p->levels] = 1;
  p->klen[p->levels] = k;
  p->ws_bytes = 2 * ((scratch + 255) / 256 * 256);
  return FX_OK;
}

int run_merge(const MergePlan& p, const uint64_t* in, int64_t nq, int64_t k, void* ws,
              float* out_dist, int64_t* out_row, hipStream_t stream, uint64_t* out_kth,
              const uint32_t* gate, int64_t gate_cap, uint32_t* count, bool zero_count) {
  const int zc = zero_count && count != nullptr && p.levels == 1 ? 1 : 0;
  const int P2 = next_pow2((int)k);
  uint64_t* bufs[2] = {reinterpret_cast<uint64_t*>(ws),
                       reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(ws) + p.ws_bytes / 2)};
  const uint64_t* cur = in;
  for (int lv = 0; lv < p.levels; ++lv) {
    const int64_t G = p.group[lv], lists = p.lists[lv], klen = p.klen[lv];
    const int64_t blocks = (lists + G - 1) / G;
    const bool fin = lv == p.levels - 1;
    uint64_t* dst = fin ? nullptr : bufs[lv & 1];
    const int rcap = P2 > k ? P2 : (int)k;
    // the input area doubles as the rank-sort output on the final level
    const int64_t sin = G * klen > k ? G * klen : k;
    const size_t smem = sizeof(MergeShared) + (size_t)rcap * 8 + (size_t)sin * 8;
    if (int rc = allow_lds((const void*)merge_kernel)) return rc;
    for (int64_t q0 = 0; q0 < nq; q0 += 65535) {
      const int64_t qn = (nq - q0) < 65535 ? (nq - q0) : 65535;
      dim3 grid((unsigned)blocks, (unsigned)qn);
      const uint64_t* src = cur + (size_t)q0 * lists * klen;
      uint64_t* dq = dst ? dst + (size_t)q0 * blocks * k : nullptr;
      float* od = out_dist ? out_dist + (size_t)q0 * k : nullptr;
      int64_t* orow = out_row ? out_row + (size_t)q0 * k : nullptr;
      uint64_t* okth = out_kth ? out_kth + q0 : nullptr;
      const uint32_t* gq = gate ? gate + (size_t)q0 * kCountStride : nullptr;
      uint32_t* cq = count != nullptr && lv == 0 ? count + (size_t)q0 * kCountStride : nullptr;
      hipLaunchKernelGGL(merge_kernel, grid, dim3(kMergeThreads), smem, stream, src, lists,
                         (int)klen, G, (int)k, P2, dq, od, orow, okth, fin ? 1 : 0, gq, gate_cap,
                         cq, zc);
      int rc = check_launch("merge_kernel");
      if (rc) return rc;
    }
    cur = dst;
  }
  return FX_OK;
}

}  // namespace fx
