// Block-wide (NT-thread, NT >= 256) selection of the k smallest 64-bit composites held
// in LDS — shared by the merge kernel and the scan kernel's epilogue.
#pragma once

#include "fx_wave.h"

namespace fx {

constexpr int kBlockThreads = 256;

struct MergeShared {
  uint32_t hist[256];
  uint32_t sh[4];
  uint32_t ctr_keep, ctr_eq;
  unsigned long long shmax, all_or, all_and;
};

// k-th smallest of s[0..m) (m > k).  start_shift: the byte holding the
// highest bit in which the entries differ (higher bytes are common to all,
// so their passes would put every entry in one bin).
template <int NT>
__device__ __forceinline__ uint64_t block_select(const uint64_t* s, int m, int k,
                                                 int start_shift, uint64_t common,
                                                 MergeShared* ms, int* quota_eq) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // the bytes above start_shift are common to every entry: they seed the prefix
  uint64_t pmask = start_shift >= 56 ? 0ull : (~0ull << (start_shift + 8));
  uint64_t prefix = common & pmask;
  uint32_t need = (uint32_t)k;
  for (int shift = start_shift; shift >= 0; shift -= 8) {
    if (tid < 256) ms->hist[tid] = 0u;
    __syncthreads();
    for (int b0 = wid * kWave; b0 < m; b0 += 4 * NT) {
      uint64_t e[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // 4 LDS reads in flight
        const int i = b0 + u * NT + lane;
        e[u] = i < m ? s[i] : kEmpty;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = b0 + u * NT + lane;
        hist_add(ms->hist, (uint32_t)(e[u] >> shift) & 255u, i < m && (e[u] & pmask) == prefix);
      }
    }
    __syncthreads();
    if (wid == 0) {
      const uint32_t h0 = ms->hist[4 * lane + 0], h1 = ms->hist[4 * lane + 1];
      const uint32_t h2 = ms->hist[4 * lane + 2], h3 = ms->hist[4 * lane + 3];
      const uint32_t sum = h0 + h1 + h2 + h3;
      const uint32_t incl = wave_incl_scan(sum, lane), excl = incl - sum;
      if (excl < need && need <= incl) {
        uint32_t c = excl, digit, below, inbin;
        if (c + h0 >= need) {
          digit = 4 * lane; below = c; inbin = h0;
        } else if (c + h0 + h1 >= need) {
          digit = 4 * lane + 1; below = c + h0; inbin = h1;
        } else if (c + h0 + h1 + h2 >= need) {
          digit = 4 * lane + 2; below = c + h0 + h1; inbin = h2;
        } else {
          digit = 4 * lane + 3; below = c + h0 + h1 + h2; inbin = h3;
        }
        ms->sh[0] = digit;
        ms->sh[1] = below;
        ms->sh[2] = inbin;
      }
      if (lane == 0) {
        ms->shmax = 0ull;
        ms->sh[3] = 0u;
      }
    }
    __syncthreads();
    const uint32_t digit = ms->sh[0], below = ms->sh[1], inbin = ms->sh[2];
    need -= below;
    prefix |= (uint64_t)digit << shift;
    pmask |= 0xffull << shift;
    if (inbin == need) {
      uint64_t mx = 0;
      for (int i = tid; i < m; i += NT) {
        const uint64_t e = s[i];
        if ((e & pmask) == prefix && e > mx) mx = e;
      }
      mx = wave_max_u64(mx);
      if (lane == 0) atomicMax(&ms->shmax, (unsigned long long)mx);
      __syncthreads();
      const uint64_t T = ms->shmax;
      int eq = 0;
      for (int i = tid; i < m; i += NT) eq += s[i] == T ? 1 : 0;
      eq = wave_sum_i(eq);
      if (lane == 0) atomicAdd(&ms->sh[3], (uint32_t)eq);
      __syncthreads();
      *quota_eq = (int)ms->sh[3];
      __syncthreads();
      return T;
    }
    __syncthreads();
  }
  *quota_eq = (int)need;
  return prefix;
}

// Reset the block reduction words (one thread), before block_or_and.
__device__ __forceinline__ void block_reset(MergeShared* ms) {
  if (threadIdx.x == 0) {
    ms->ctr_keep = 0u;
    ms->ctr_eq = 0u;
    ms->all_or = 0ull;
    ms->all_and = ~0ull;
  }
}

// Fold a thread's OR/AND of its entries into ms (call after block_reset and a
// barrier; a barrier must follow before reading ms->all_or / all_and).
__device__ __forceinline__ void block_or_and(uint64_t v_or, uint64_t v_and, MergeShared* ms) {
#pragma unroll
  for (int msk = 32; msk >= 1; msk >>= 1) {
    v_or |= shfl_xor_u64(v_or, msk);
    v_and &= shfl_xor_u64(v_and, msk);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicOr(&ms->all_or, (unsigned long long)v_or);
    atomicAnd(&ms->all_and, (unsigned long long)v_and);
  }
}

// Keep the k smallest of s[0..m) (m > k; all_or/all_and ready in ms): writes
// exactly k entries, in no particular order, to dst[0..k) (LDS or global).
template <int NT>
__device__ __forceinline__ void block_keep_k(const uint64_t* s, int m, int k, uint64_t* dst,
                                             MergeShared* ms) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t diff = ms->all_or ^ ms->all_and;
  const int start_shift = diff ? (63 - __clzll((long long)diff)) / 8 * 8 : 0;
  int quota;
  const uint64_t T = block_select<NT>(s, m, k, start_shift, ms->all_and, ms, &quota);
  const uint64_t ltmask = (1ull << lane) - 1ull;
  for (int base = wid * kWave; base < m; base += NT) {
    const int i = base + lane;
    const bool in_range = i < m;
    const uint64_t e = in_range ? s[i] : kEmpty;
    const bool lt = in_range && e < T;
    const bool eq = in_range && e == T;
    const uint64_t beq = __ballot(eq);
    uint32_t eqbase = 0;
    if (beq) {
      if (lane == 0) eqbase = atomicAdd(&ms->ctr_eq, (uint32_t)__popcll(beq));
      eqbase = __shfl(eqbase, 0);
    }
    const bool keep = lt || (eq && (int)(eqbase + __popcll(beq & ltmask)) < quota);
    const uint64_t bk = __ballot(keep);
    if (bk) {
      uint32_t pos = 0;
      if (lane == 0) pos = atomicAdd(&ms->ctr_keep, (uint32_t)__popcll(bk));
      pos = __shfl(pos, 0);
      if (keep) dst[pos + __popcll(bk & ltmask)] = e;
    }
  }
}

}  // namespace fx
