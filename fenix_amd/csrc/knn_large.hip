// Top-k for k beyond the fused path (k > 1024): every distance, then a radix
// sort of (distance, row) composites.
//
// The reference accepts any maxval (src/fenix/io/index/index.py:165-168:
// pc.select_k_unstable(data, maxval, ...) over the whole table), so a drop-in
// must too.  The fused scan keeps per-wave candidate lists in LDS, which caps k
// at 1024; above it the scan runs in distance mode (the same kernel, one f32
// per row to HBM: +1/D of the corpus bytes), a small kernel turns distances
// into composites (masked rows -> kEmpty), hipcub's onesweep radix sort orders
// each query's composites, and the first k are decoded.  Same ordering
// contract and tie-break as the fused path; cost ~ one extra pass over n keys.
#include <hipcub/hipcub.hpp>

#include "fx_internal.h"

namespace fx {

namespace {

size_t align256(size_t v) { return (v + 255) / 256 * 256; }

__global__ void dist_keys_kernel(const float* __restrict__ dist, int64_t n, int64_t row_base,
                                 const uint32_t* __restrict__ mask,
                                 const int32_t* __restrict__ rows, uint64_t* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t q = blockIdx.y;
  if (i >= n) return;
  const int64_t r = rows != nullptr ? (int64_t)rows[i] : i;
  const bool valid = mask == nullptr || ((mask[r >> 5] >> (r & 31)) & 1u);
  keys[q * n + i] = valid ? make_comp(dist[q * n + i], (uint32_t)(row_base + r)) : kEmpty;
}

__global__ void decode_kernel(const uint64_t* __restrict__ sorted, int64_t len, int64_t k,
                              float* __restrict__ out_dist, int64_t* __restrict__ out_row) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t q = blockIdx.y;
  if (j >= k) return;
  const uint64_t e = j < len ? sorted[q * len + j] : kEmpty;
  out_dist[q * k + j] = e == kEmpty ? __builtin_nanf("") : key_float((uint32_t)(e >> 32));
  out_row[q * k + j] = e == kEmpty ? -1 : (int64_t)(e & 0xffffffffull);
}

size_t sort_temp_bytes(int64_t len) {
  size_t t = 0;
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, t, (const uint64_t*)nullptr,
                                          (uint64_t*)nullptr, (int)len, 0, 64, (hipStream_t)0);
  return t;
}

// sort each query's `len` keys (one onesweep sort per query) and decode k
int sort_decode(uint64_t* keys, uint64_t* sorted, void* temp, size_t temp_bytes, int64_t nq,
                int64_t len, int64_t k, float* out_dist, int64_t* out_row, hipStream_t st) {
  for (int64_t q = 0; q < nq; ++q) {
    size_t t = temp_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortKeys(temp, t, keys + q * len, sorted + q * len,
                                                     (int)len, 0, 64, st);
    if (e != hipSuccess) {
      set_error("radix sort: %s", hipGetErrorString(e));
      return FX_EHIP;
    }
  }
  for (int64_t q0 = 0; q0 < nq; q0 += 65535) {
    const int64_t qn = (nq - q0) < 65535 ? (nq - q0) : 65535;
    hipLaunchKernelGGL(decode_kernel, dim3((unsigned)((k + 255) / 256), (unsigned)qn), dim3(256),
                       0, st, sorted + q0 * len, len, k, out_dist + q0 * k, out_row + q0 * k);
    int rc = check_launch("decode_kernel");
    if (rc) return rc;
  }
  return FX_OK;
}

}  // namespace

LargeLayout plan_large(int64_t n, int64_t nq) {
  LargeLayout l;
  size_t off = 0;
  l.off_dist = off;
  off += align256((size_t)nq * n * 4);
  l.off_keys = off;
  off += align256((size_t)nq * n * 8);
  l.off_sorted = off;
  off += align256((size_t)nq * n * 8);
  l.temp_bytes = sort_temp_bytes(n);
  l.off_temp = off;
  off += align256(l.temp_bytes);
  l.total = off;
  return l;
}

int large_scan(const ScanPlan& p, ScanArgs a, int64_t nq, const LargeLayout& l, char* ws,
               hipStream_t st) {
  float* dist = reinterpret_cast<float*>(ws + l.off_dist);
  a.mode = kModeDist;
  a.k = 1;
  const int64_t n = a.n;
  const float* q0p = a.q;
  for (int64_t q0 = 0; q0 < nq; q0 += 65535) {
    const int64_t qn = (nq - q0) < 65535 ? (nq - q0) : 65535;
    a.q = q0p + (size_t)q0 * a.d;
    a.out_dist = dist + (size_t)q0 * n;
    int rc = launch_scan(p, a, qn, st);
    if (rc) return rc;
  }
  uint64_t* keys = reinterpret_cast<uint64_t*>(ws + l.off_keys);
  for (int64_t q0 = 0; q0 < nq; q0 += 65535) {
    const int64_t qn = (nq - q0) < 65535 ? (nq - q0) : 65535;
    hipLaunchKernelGGL(dist_keys_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)qn),
                       dim3(256), 0, st, dist + q0 * n, n, a.row_base, a.mask, a.rows,
                       keys + q0 * n);
    int rc = check_launch("dist_keys_kernel");
    if (rc) return rc;
  }
  return FX_OK;
}

int large_reduce(int64_t n, int64_t nq, int64_t k, const LargeLayout& l, char* ws,
                 float* out_dist, int64_t* out_row, hipStream_t st) {
  return sort_decode(reinterpret_cast<uint64_t*>(ws + l.off_keys),
                     reinterpret_cast<uint64_t*>(ws + l.off_sorted), ws + l.off_temp,
                     l.temp_bytes, nq, n, k, out_dist, out_row, st);
}

// fx_topk_merge above the merge kernels' limit: composites already in
// ws + off_keys ([nq][len]); sort and decode.
int large_merge(int64_t nq, int64_t len, int64_t k, const LargeLayout& l, char* ws,
                float* out_dist, int64_t* out_row, hipStream_t st) {
  return large_reduce(len, nq, k, l, ws, out_dist, out_row, st);
}

}  // namespace fx
