// extern "C" entry points declared in include/fenix_knn.h, plus the error and
// device-property helpers the kernels' planners use.
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <map>
#include <set>
#include <tuple>
#include <vector>
#include <mutex>
#include <utility>

#include "fx_internal.h"

namespace fx {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return FX_EHIP;
  }
  return FX_OK;
}

static std::mutex g_mu;

// ----------------------------------------------------------------- options --
static const char* const kOptNames[kOptCount] = {
    "batched", "batch_min_queries", "batch_cap", "batch_sample_ratio",
    "force_fallback", "scan_interleave", "q8_dma", "filter_image", "batch_ub_test",
    "single_query_image", "i8_max_k", "img6", "img8", "i8_sample_ratio", "i8_grow_ratio",
    "select_prune"};
static std::atomic<int64_t> g_opts[kOptCount] = {{1}, {2}, {0}, {0}, {0}, {-1}, {1}, {8}, {1}, {1},
                                                 {1024}, {1}, {1}, {8}, {16}, {1}};

int64_t option(Option o) { return g_opts[o].load(std::memory_order_relaxed); }

static int option_index(const char* name) {
  if (name == nullptr) return -1;
  for (int i = 0; i < kOptCount; ++i)
    if (strcmp(name, kOptNames[i]) == 0) return i;
  return -1;
}

#ifdef FX_DIAG_BUILD
int diag_env(const char* name, int dflt) {
  const char* env = getenv(name);
  return env != nullptr ? atoi(env) : dflt;
}
#endif

// host-blocking synchronisations performed (fx_host_sync_count); searches
// perform none, and any added one must go through host_sync
static std::atomic<uint64_t> g_host_syncs{0};

int device_cus(int* out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) {
    set_error("hipGetDevice: %s", hipGetErrorString(e));
    return FX_EHIP;
  }
  static std::map<int, int> cache;
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = cache.find(dev);
  if (it != cache.end()) {
    *out = it->second;
    return FX_OK;
  }
  int cus = 0;
  e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) {
    set_error("hipDeviceGetAttribute: %s", hipGetErrorString(e));
    return FX_EHIP;
  }
  cache[dev] = cus;
  *out = cus;
  return FX_OK;
}

// The dynamic-LDS limit above 64 KB is a per-device function attribute: set
// it once per (device, kernel), so a table sharded over several devices can
// launch the same kernel on each of them.
int allow_lds(const void* fn) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) {
    set_error("hipGetDevice: %s", hipGetErrorString(e));
    return FX_EHIP;
  }
  static std::set<std::pair<int, const void*>> done;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!done.insert(std::make_pair(dev, fn)).second) return FX_OK;
  // the dynamic share of the 160 KB: whatever the kernel's static __shared__
  // variables leave
  hipFuncAttributes at = {};
  e = hipFuncGetAttributes(&at, fn);
  if (e != hipSuccess) {
    done.erase(std::make_pair(dev, fn));
    set_error("hipFuncGetAttributes: %s", hipGetErrorString(e));
    return FX_EHIP;
  }
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                          160 * 1024 - (int)at.sharedSizeBytes);
  if (e != hipSuccess) {
    done.erase(std::make_pair(dev, fn));
    set_error("hipFuncSetAttribute(MaxDynamicSharedMemorySize): %s", hipGetErrorString(e));
    return FX_EHIP;
  }
  return FX_OK;
}

int kernel_occupancy(const void* fn, int block, size_t smem, int* out) {
  if (smem > 64 * 1024) {
    int rc = allow_lds(fn);
    if (rc) return rc;
  }
  int dev = 0;
  hipError_t e0 = hipGetDevice(&dev);
  if (e0 != hipSuccess) {
    set_error("hipGetDevice: %s", hipGetErrorString(e0));
    return FX_EHIP;
  }
  static std::map<std::tuple<int, const void*, size_t>, int> cache;
  std::lock_guard<std::mutex> lk(g_mu);
  auto key = std::make_tuple(dev, fn, smem);
  auto it = cache.find(key);
  if (it != cache.end()) {
    *out = it->second;
    return FX_OK;
  }
  int nb = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, block, smem);
  if (e != hipSuccess) {
    set_error("hipOccupancyMaxActiveBlocksPerMultiprocessor: %s", hipGetErrorString(e));
    return FX_EHIP;
  }
  cache[key] = nb;
  *out = nb;
  return FX_OK;
}

static size_t align256(size_t v) { return (v + 255) / 256 * 256; }

static int validate(int64_t n, int64_t d, int dtype, int64_t nq, int metric) {
  if (n < 1 || d < 1 || nq < 1) {
    set_error("invalid shape n=%lld d=%lld nq=%lld", (long long)n, (long long)d, (long long)nq);
    return FX_EINVAL;
  }
  if (d > (1 << 20)) {
    set_error("d=%lld too large", (long long)d);
    return FX_EUNSUPPORTED;
  }
  if (dtype != FX_DTYPE_F32 && dtype != FX_DTYPE_F16) {
    set_error("unsupported dtype %d", dtype);
    return FX_EINVAL;
  }
  if (metric < FX_METRIC_L2 || metric > FX_METRIC_COS) {
    set_error("unsupported metric %d", metric);
    return FX_EINVAL;
  }
  return FX_OK;
}

static constexpr int64_t kMaxK = 1024;  // fused path; larger k: knn_large.hip
static constexpr int64_t kLargeMaxK = 0x7fffffffll;

// ---------------------------------------------------------------- batched --
//
// Batched queries (nq >= kBatchMinQ, f32) run the MFMA kernel of knn_batch.hip
// in phases over growing row samples (L2: the GEMM gives |x|^2+|q|^2-2x.q,
// rows pass on a rigorous fp32 lower bound and every appended candidate is
// rescored exactly before any threshold or result is taken):
//   phase 0: a sample of <= cap rows, no threshold -> every (row, query) kept;
//   phase i: a sample ~cap/(4k) times larger, threshold = the k-th composite
//            of phase i-1 (an upper bound of the global k-th: the k-th of any
//            row subset is), so it keeps ~cap/4 candidates per query;
//   last:    every row with the last threshold -> final select.
// A query whose final candidates overflow `cap` is recomputed exactly by the
// single-query scan, gated on the device (fx_knn_reduce: no host sync).
static constexpr int64_t kListLen = 4096;  // candidate buffer viewed as lists
// int8 filter image (filter_phases_i8): the final pass's sample F1 takes
// every r1-th tile, the samples before it grow by r2 (options
// "i8_sample_ratio", default 8, and "i8_grow_ratio", default 16)

struct BatchLayout {
  int64_t cap = 0, tiles = 0, nq_pad = 0;
  int nphases = 0;
  bool filter = false;  // fp16-MFMA filter + exact rescoring (knn_filter.hip)
  bool img8 = false;    // planned for an int8 filter image (filter_phases_i8)
  int dq = 0;
  int64_t start[16], stride[16], num[16];
  MergePlan merge;
  size_t off_qnorm, off_thr, off_count, off_cand, off_merge, off_cand_ub, off_qh, off_qinfo,
      off_topd, off_topr, off_prune, total;
};

// The fp16-MFMA filter (knn_filter.hip).  Diagnostic builds keep the
// rejected fp32-MFMA batch kernel (knn_batch.hip) behind FX_BATCH_FILTER=0.
static bool use_filter() { return diag_env("FX_BATCH_FILTER", 1) != 0; }

// A single query over an f32 corpus of at least this many bytes takes the
// batched path when an int8 filter image is supplied (the *_img8 entry
// points, option "single_query_image"): 10M x 768 1.41 vs 4.34 ms; the
// filter path's fixed cost (~0.25 ms of small launches) loses below ~2.4 GB
static constexpr int64_t kSingleImageMinBytes = (int64_t)4 << 30;
// Int8 images serve k <= option "i8_max_k" (1 024 = kMaxK, every k the
// filter plans).  Round 3's 64 K slots overflowed at k = 1 000 (6.25M x 1536
// fp16 IP, profiles/r03_f16_int8_image.log); with the 4x buffer (256 K slots
// at k = 1 000), the pruned selects (select_kernel MODE 3) and the shared LDS
// append segments, 60 single queries (normal, near, clustered corpus) kept
// 94-122 K candidates, none overflowed, 1.67 vs 2.84 ms for the exact scan,
// bit-identical (profiles/r06_k1000_sweep*.json); batches at k 300-1 000 are
// faster too (profiles/r06_kbatch_i8_max_k.jsonl).
static int64_t i8_max_k() { return option(kOptI8MaxK); }

static bool use_batched(int64_t nq, int dtype, int metric, int64_t d, bool aligned, int64_t n,
                        bool img8, int64_t k) {
  if (option(kOptBatched) == 0) return false;
  // 2 queries: 6.5 ms vs 2 x 4.5 ms (10Mx768); "batch_min_queries" = 1 also
  // sends every single query through the filter
  int64_t min_q = option(kOptBatchMinQ) >= 1 ? option(kOptBatchMinQ) : 2;
  if (nq == 1 && img8 && k <= i8_max_k() && option(kOptSingleImage) != 0 && d % 8 == 0 &&
      n * d * (dtype == FX_DTYPE_F32 ? 4 : 2) >= kSingleImageMinBytes)
    min_q = 1;
  if (!use_filter()) min_q = 8;  // the fp32-MFMA kernel breaks even with scans at ~8 queries
  if (nq < min_q || !aligned) return false;
  // the rescoring repeats the scan's 16-B slot order: f32 rows need d % 4 == 0,
  // f16 rows d % 8 == 0 (and the fp16 filter: the fp32-MFMA kernel reads f32 only)
  if (dtype == FX_DTYPE_F32) return d % 4 == 0;
  return dtype == FX_DTYPE_F16 && d % 8 == 0 && use_filter();
}

static int plan_phases(BatchLayout* b, int64_t tr, int64_t r);

static int plan_batched(int64_t n, int64_t d, int dtype, int64_t nq, int64_t k, BatchLayout* b,
                        bool img8) {
  b->filter = use_filter();
  b->img8 = img8 && b->filter;
  const int64_t tr = b->filter ? filter_tile_rows(dtype) : batch_tile_rows();
  b->cap = 64 * k > 16384 ? 64 * k : 16384;
  // int8 images: 4x the buffer.  Their bounds keep whole clusters of a
  // clustered corpus against a generic query (10M x 768, x + 10 x0 per
  // 1 000 rows, 256 cosine queries: median 10 K, largest 33 K candidates);
  // every consumer reads only the count it was given (select_kernel streams
  // any count), so the larger buffer costs memory, not time
  if (b->img8) b->cap *= 4;
  if (option(kOptBatchCap) >= 16 * k) b->cap = option(kOptBatchCap);  // test: small buffers
  b->cap = (b->cap + kListLen - 1) / kListLen * kListLen;
  b->tiles = (n + tr - 1) / tr;
  // nested samples: phase i scans every stride_i-th tile, each stride a
  // multiple of the next, so every sample contains the previous one and has
  // at least k rows under the previous threshold; ~cap/4 appends per query.
  int64_t r = b->cap / (4 * k);  // >= 16 for k <= 1024
  {  // test switch: denser samples (never sparser)
    const int64_t v = option(kOptBatchRatio);
    if (v >= 2 && v < r) r = v;
  }
  int rc = plan_phases(b, tr, r);
  if (rc) return rc;
  rc = plan_merge(nq, b->cap / kListLen, kListLen, k, &b->merge);
  if (rc) return rc;
  size_t off = 0;
  b->off_qnorm = off;
  off += align256((size_t)nq * 4);
  b->off_thr = off;
  off += align256((size_t)nq * 8);
  b->off_count = off;
  off += align256((size_t)nq * 4 * kCountStride);
  b->off_cand = off;
  off += align256((size_t)nq * b->cap * 8);
  b->off_merge = off;
  off += align256(b->merge.ws_bytes);
  if (b->filter) {
    b->dq = filter_dq((int)d);
    b->nq_pad = (nq + filter_query_pad(nq) - 1) / filter_query_pad(nq) * filter_query_pad(nq);
    b->off_cand_ub = off;
    off += align256((size_t)nq * b->cap * 8);
    // fp16 query tiles, or int8 ones padded to 256 queries (int8 filter images)
    const size_t q16 = (size_t)b->nq_pad * b->dq * 2, q8 = (size_t)((nq + 255) / 256 * 256) * b->dq;
    b->off_qh = off;
    off += align256(q16 > q8 ? q16 : q8);
    b->off_qinfo = off;
    off += align256((size_t)nq * 16);
    // the k best candidates by upper bound (int8 images: exact thresholds)
    b->off_topd = off;
    off += align256((size_t)nq * k * 4);
    b->off_topr = off;
    off += align256((size_t)nq * k * 8);
  }
  // the selects' prune scratch (int8 plans at large k: select_prune_lists)
  b->off_prune = off;
  if (b->img8) off += align256(select_prune_bytes(nq, k, b->cap));
  b->total = off;
  return FX_OK;
}

// Nested row samples of the batched phases: phase i scans every stride_i-th
// tile of tr rows, each stride a multiple r of the next, the first at most
// cap rows, the last every tile.
// The int8 image's plan (filter_phases_i8).  The image stores its rows in a
// permuted order (image8_perm: a Weyl sequence over the corpus), so any
// PREFIX of its tiles is an equidistributed sample of the corpus: the
// samples are nested prefixes, read as contiguous runs.  The last sample F1
// holds ceil(tiles / r1) tiles (F2 reads the rest), the ones before it
// shrink by r2 (their appends stay far below cap: about r2 k upper bounds
// per query), the first holds at most cap rows.  10M x 768, r1 = 8, r2 = 16:
// 20, 306, 4 883 tiles, then F2's 34 180.
static int plan_phases_i8(BatchLayout* b, int64_t tr, int64_t r1, int64_t r2) {
  int64_t nums[16];
  int m = 0;
  nums[m++] = b->tiles;
  int64_t r = r1;
  while (nums[m - 1] * tr > b->cap) {
    if (m >= 15) {
      set_error("batched sampling plan too deep");
      return FX_EUNSUPPORTED;
    }
    nums[m] = (nums[m - 1] + r - 1) / r;
    ++m;
    r = r2;
  }
  b->nphases = m;
  for (int i = 0; i < m; ++i) {
    b->num[i] = nums[m - 1 - i];
    b->start[i] = 0;
    b->stride[i] = 1;
  }
  return FX_OK;
}

static int plan_phases(BatchLayout* b, int64_t tr, int64_t r) {
  int64_t strides[16];
  int m = 0;
  strides[m++] = 1;
  while ((b->tiles + strides[m - 1] - 1) / strides[m - 1] * tr > b->cap) {
    if (m >= 15) {
      set_error("batched sampling plan too deep");
      return FX_EUNSUPPORTED;
    }
    strides[m] = strides[m - 1] * r;
    ++m;
  }
  b->nphases = m;
  for (int i = 0; i < m; ++i) {
    const int64_t st = strides[m - 1 - i];
    b->stride[i] = st;
    b->start[i] = 0;
    b->num[i] = (b->tiles + st - 1) / st;
  }
  return FX_OK;
}

struct SearchLayout {
  ScanPlan scan;
  MergePlan merge;
  size_t lists_bytes, total;
  bool large = false;  // k > kMaxK: distance-mode scan + radix sort (knn_large.hip)
  LargeLayout lg;
  bool batched;
  BatchLayout batch;
  size_t single_off;   // batched: workspace of the overflow fallback
  int64_t fb_queries;  // batched: queries per fallback round (scan + merge over fb_queries)
};

static int plan_single(int64_t n, int64_t d, int dtype, int64_t nq, int64_t k, int metric,
                       bool aligned, SearchLayout* s) {
  int rc = plan_scan(n, d, dtype, k, metric, aligned, &s->scan);
  if (rc) return rc;
  rc = plan_merge(nq, s->scan.nlists, k, k, &s->merge);
  if (rc) return rc;
  s->lists_bytes = align256((size_t)nq * s->scan.nlists * k * 8);
  s->total = s->lists_bytes + s->merge.ws_bytes;
  s->batched = false;
  return FX_OK;
}

static int plan_large_search(int64_t n, int64_t d, int dtype, int64_t nq, int metric,
                             bool aligned, SearchLayout* s) {
  int rc = plan_scan(n, d, dtype, 1, metric, aligned, &s->scan);
  if (rc) return rc;
  s->large = true;
  s->batched = false;
  s->lg = plan_large(n, nq);
  s->lists_bytes = 0;
  s->total = s->lg.total;
  return FX_OK;
}

// The overflow fallback of the batched path runs the single-query plan over
// rounds of fq queries; its candidate lists take at most this many bytes.
static constexpr size_t kFallbackListBytes = (size_t)256 << 20;

// Its scan takes at most kFallbackBlocks blocks per query: the gated launch
// covers every query of a round, and an empty block still occupies its CU's
// LDS while it starts and exits (256 blocks x 256 queries of 10M x 768: 99 us
// with nothing to do; 16 per query: a few us, and an overflowing query still
// streams its rows from 16 CUs).
// Small batches spread the same total over more workgroups per query (4 096
// workgroups in all, at least 16 per query): a single query that overflows is
// rescanned at the full scan's width (256 workgroups, ~4.4 ms for 10M x 768)
// instead of by 16 CUs (~38 ms).
static constexpr int64_t kFallbackBlocks = 16;
static constexpr int64_t kFallbackTotalBlocks = 4096;

static int plan_fallback(int64_t n, int64_t d, int dtype, int64_t nq, int64_t k, int metric,
                         bool aligned, SearchLayout* s, int64_t* fq) {
  int rc = plan_scan(n, d, dtype, k, metric, aligned, &s->scan);
  if (rc) return rc;
  const int64_t per_q = kFallbackTotalBlocks / (nq > 0 ? nq : 1);
  limit_scan_blocks(&s->scan, n, per_q > kFallbackBlocks ? per_q : kFallbackBlocks);
  const size_t per_query = (size_t)s->scan.nlists * k * 8;
  int64_t f = (int64_t)(kFallbackListBytes / (per_query > 0 ? per_query : 1));
  if (f > nq) f = nq;
  if (f > 65535) f = 65535;
  if (f < 1) f = 1;
  *fq = f;
  rc = plan_merge(f, s->scan.nlists, k, k, &s->merge);
  if (rc) return rc;
  s->lists_bytes = align256((size_t)f * s->scan.nlists * k * 8);
  s->total = s->lists_bytes + s->merge.ws_bytes;
  s->batched = false;
  return FX_OK;
}

// img8: the call supplies an int8 filter image (single queries may take
// the batched path, use_batched); the reduce must plan with the same flag
static int plan_search(int64_t n, int64_t d, int dtype, int64_t nq, int64_t k, int metric,
                       bool aligned, SearchLayout* s, bool img8 = false) {
  if (k > kMaxK) return plan_large_search(n, d, dtype, nq, metric, aligned, s);
  if (!use_batched(nq, dtype, metric, d, aligned, n, img8, k)) {
    return plan_single(n, d, dtype, nq, k, metric, aligned, s);
  }
  // the single-query plan over fb_queries queries serves overflowing queries
  int64_t fq = 1;
  int rc = plan_fallback(n, d, dtype, nq, k, metric, aligned, s, &fq);
  if (rc) return rc;
  const size_t single_total = s->total;
  rc = plan_batched(n, d, dtype, nq, k, &s->batch,
                    img8 && k <= i8_max_k() && d % 8 == 0 &&
                        (dtype == FX_DTYPE_F32 || dtype == FX_DTYPE_F16));
  if (rc) return rc;
  s->batched = true;
  s->fb_queries = fq;
  s->single_off = s->batch.total;
  s->total = s->batch.total + single_total;
  return FX_OK;
}


// The fallback scan's arguments: top-k lists into ws, each workgroup gated
// on its query's count (> gate_cap: recompute)
static ScanArgs fallback_args(const SearchLayout& s, const void* corpus, int64_t n, int64_t d,
                              int64_t row_base, int64_t k, const uint32_t* mask, int64_t gate_cap,
                              char* ws) {
  ScanArgs a = {};
  a.X = corpus;
  a.n = n;
  a.d = (int)d;
  a.row_base = row_base;
  a.mask = mask;
  a.rows_per_block = s.scan.rows_per_block;
  a.k = (int)k;
  a.cap = s.scan.cap;
  a.qbytes = s.scan.qbytes;
  a.mode = kModeTopk;
  a.out_lists = reinterpret_cast<uint64_t*>(ws);
  a.gate_cap = gate_cap;
  return a;
}

// The fallback's gated scan alone over all nq queries (s.fb_queries >= nq):
// per overflowing query nlists lists of k composites at *lists, [nq][nlists k]
static int fallback_scan(const SearchLayout& s, const void* corpus, int64_t n, int64_t d,
                         int64_t row_base, const float* queries, int64_t nq, int64_t k,
                         const uint32_t* mask, const uint32_t* count, int64_t gate_cap, char* ws,
                         hipStream_t st, const uint64_t** lists) {
  ScanArgs a = fallback_args(s, corpus, n, d, row_base, k, mask, gate_cap, ws);
  a.q = queries;
  a.gate = count;
  *lists = a.out_lists;
  return launch_scan(s.scan, a, nq, st);
}

// Batched-path fallback: the exact single-query scan + merge of every query
// whose final candidates overflowed the buffer (count[q] > gate_cap; all of
// them when gate_cap < 0), in rounds of s.fb_queries.  Decided on the device:
// each workgroup reads its query's count and returns at once when it did not
// overflow, so nothing waits for the host; the merge writes only the
// recomputed queries' results.
static int fallback_search(const SearchLayout& s, const void* corpus, int dtype, int64_t n,
                           int64_t d, int64_t row_base, const float* queries, int64_t nq,
                           int metric, int64_t k, const uint32_t* mask, const uint32_t* count,
                           int64_t gate_cap, char* ws, float* out_dist, int64_t* out_row,
                           hipStream_t st) {
  (void)dtype;
  (void)metric;
  ScanArgs a = fallback_args(s, corpus, n, d, row_base, k, mask, gate_cap, ws);
  for (int64_t q0 = 0; q0 < nq; q0 += s.fb_queries) {
    const int64_t qn = (nq - q0) < s.fb_queries ? (nq - q0) : s.fb_queries;
    a.q = queries + (size_t)q0 * d;
    a.gate = count + (size_t)q0 * kCountStride;
    int rc = launch_scan(s.scan, a, qn, st);
    if (rc) return rc;
    rc = run_merge(s.merge, a.out_lists, qn, k, ws + s.lists_bytes, out_dist + (size_t)q0 * k,
                   out_row + (size_t)q0 * k, st, nullptr, a.gate, gate_cap);
    if (rc) return rc;
  }
  return FX_OK;
}

// fp16 filter phases (knn_filter.hip).  Sampling phases append the UPPER
// bound of every row whose lower bound reaches the threshold; the k-th upper
// bound of any row subset bounds the global k-th distance from above, so it is
// the next phase's threshold.  The final phase (every row) appends lower and
// upper bounds; the k-th upper bound among its candidates is a tighter
// threshold, and only candidates whose lower bound reaches it are rescored
// exactly (the rest are dropped unread).  fx_knn_reduce then selects the top k
// of the exact keys and recomputes overflowing queries.
// With an fp16 filter image of an f32 corpus (fx_filter_image) the phases
// stream the image (half the bytes) and the rescoring reads the f32 rows.
//
// An int8 filter image (fx_filter_image8) gives bounds ~30x wider than fp16
// (per-row 8-bit quantization, see knn_filter.hip "int8 filter image"), so a
// k-th upper bound sits well above the k-th distance: after the last two
// phases the k candidates with the smallest upper bounds are rescored exactly
// (launch_exact_kth) and their largest exact composite becomes the threshold
// (k scan distances lie at or below it), and the samples grow by
// kI8SampleRatio per phase, which keeps the appends below cap/4 per query
// (10M x 768 cosine, 256 queries: ~2.5 K, 6 K, 10 K, 4 K per phase).
static int filter_phases(const BatchLayout& b, const void* X, int dtype, const void* image,
                         const float* rowinfo, bool img8, int64_t n, int64_t d, int64_t row_base,
                         const float* Q, int64_t nq, int metric, int64_t k,
                         const uint32_t* mask, char* w, hipStream_t st) {
  float* qnorm = reinterpret_cast<float*>(w + b.off_qnorm);
  uint64_t* thr = reinterpret_cast<uint64_t*>(w + b.off_thr);
  uint32_t* count = reinterpret_cast<uint32_t*>(w + b.off_count);
  uint64_t* cand = reinterpret_cast<uint64_t*>(w + b.off_cand);
  uint64_t* cand_ub = reinterpret_cast<uint64_t*>(w + b.off_cand_ub);
  uint16_t* qh = reinterpret_cast<uint16_t*>(w + b.off_qh);
  float* qinfo = reinterpret_cast<float*>(w + b.off_qinfo);
  const int64_t nq_pad8 = (nq + 255) / 256 * 256;
  int rc = img8 ? launch_qprep8(Q, nq, nq_pad8, (int)d, b.dq, metric,
                                reinterpret_cast<int8_t*>(qh), qinfo, st)
                : launch_qprep(Q, nq, b.nq_pad, (int)d, b.dq, metric, qh, qinfo, st);
  if (rc) return rc;
  if (metric == FX_METRIC_COS) {  // the scan's max(|q|, 1e-12) for the rescoring
    rc = launch_qnorm(Q, nq, (int)d, qnorm, st, 0);
    if (rc) return rc;
  }
  hipError_t e = hipMemsetAsync(thr, 0xFF, (size_t)nq * 8, st);
  // a one-level threshold merge resets the counts it read, so only the first
  // phase needs a fill (each fill is a ~5 us launch)
  const bool merge_zeroes = b.merge.levels == 1;
  for (int ph = 0; ph < b.nphases && e == hipSuccess; ++ph) {
    const bool last = ph + 1 == b.nphases;
    // (the lists are read up to count only: no fill of the candidate buffers)
    if (ph == 0 || !merge_zeroes) e = hipMemsetAsync(count, 0, (size_t)nq * 4 * kCountStride, st);
    if (e != hipSuccess) break;
    FilterArgs a = {};
    a.X = image != nullptr ? image : X;
    a.dtype = image != nullptr ? FX_DTYPE_F16 : dtype;
    a.rowinfo = image != nullptr ? rowinfo : nullptr;
    a.n = n;
    a.d = (int)d;
    a.row_base = row_base;
    a.Qh = qh;
    a.dq = b.dq;
    a.qstride = img8 ? nq_pad8 : b.nq_pad;
    a.img8 = img8 ? 1 : 0;
    a.all_pass = ph == 0 ? 1 : 0;  // (thr was just filled with the empty key)
    // sampling phases need only the k smallest upper bounds of their rows:
    // the k rows behind the previous threshold are in this (nested) sample
    // with upper bounds at or below it, so no row whose upper bound exceeds
    // it is among them (option "batch_ub_test" = 0: the lower-bound test)
    a.ub_test = ph > 0 && !last && option(kOptBatchUbTest) != 0 ? 1 : 0;
    a.qinfo = qinfo;
    a.nq = nq;
    a.mask = mask;
    a.tile_start = b.start[ph];
    a.tile_stride = b.stride[ph];
    a.num_tiles = b.num[ph];
    a.thr = thr;
    a.count = count;
    a.cand = cand;
    a.cand_ub = last ? cand_ub : nullptr;
    a.cap = (int)b.cap;
    a.diag = diag_env("FX_FILTER_DIAG", 0);
    rc = launch_filter(a, metric, st);
    if (rc) return rc;
    // int8 images, the last two phases: the exact distances of the k best
    // upper bounds give the next threshold (earlier, small samples: the k-th
    // upper bound, like fp16; their appends stay far below cap)
    if (img8 && ph + 2 >= b.nphases) {
      float* topd = reinterpret_cast<float*>(w + b.off_topd);
      int64_t* topr = reinterpret_cast<int64_t*>(w + b.off_topr);
      rc = run_merge(b.merge, last ? cand_ub : cand, nq, k, w + b.off_merge, topd, topr, st,
                     nullptr, nullptr, 0, count, !last);
      if (rc) return rc;
      rc = launch_exact_kth(X, dtype, n, (int)d, row_base, Q, qnorm, nq, (int)k, topr, metric,
                            thr, st);
      if (rc) return rc;
      continue;
    }
    // the k-th upper bound of this phase's candidates: next threshold
    rc = run_merge(b.merge, last ? cand_ub : cand, nq, k, w + b.off_merge, nullptr, nullptr, st,
                   thr, nullptr, 0, count, !last);
    if (rc) return rc;
  }
  if (e != hipSuccess) {
    set_error("batched memset: %s", hipGetErrorString(e));
    return FX_EHIP;
  }
  return launch_rescore(X, dtype, n, (int)d, row_base, Q, qnorm, nq, count, cand, (int)b.cap,
                        metric, thr, st);
}

// The int8 image's phases (fx_filter_image8; rows in image8_perm order, so
// every sample is equidistributed over the corpus):
//   sampling phases 0 .. m-3: phase 0 appends every pair of its <= cap rows,
//     later ones the upper bounds at or below the previous threshold; the k-th
//     upper bound is the next threshold, and after phase m-3 the exact
//     distances of the k best upper bounds (launch_exact_kth) set it;
//   F1 (phase m-2, the last sample's prefix of tiles): every pair whose lower bound
//     reaches that threshold, appended with both bounds into the final
//     candidate buffer; the exact k-th of its k best upper bounds is the
//     next, much tighter threshold;
//   overflow gate: F1's candidates under the new threshold, scaled to the
//     tiles left, predict the final count; a query predicted past cap skips
//     the final pass and goes to the exact scan (fx_knn_reduce's fallback);
//   F2 (phase m-1): the tiles after F1's prefix, lower bound against the
//     new threshold, appended after F1's candidates.  Each image row is
//     read once by F1 or F2 (the sampling phases re-read 1/r1 (1/r2 + ...)
//     of them);
//   the exact k-th of all candidates' k best upper bounds is the final
//     threshold (batches of more than kI8RescoreAllMaxQ queries; smaller ones
//     keep F1's), and the candidates whose lower bound reaches it are
//     rescored exactly (launch_rescore), fx_knn_reduce selects the top k.
static constexpr int64_t kI8RescoreAllMaxQ = 2;

static int filter_phases_i8(const BatchLayout& b, const void* X, int dtype, const void* image,
                            const float* rowinfo, int64_t n, int64_t d, int64_t row_base,
                            const float* Q, int64_t nq, int metric, int64_t k,
                            const uint32_t* mask, char* w, hipStream_t st) {
  float* qnorm = reinterpret_cast<float*>(w + b.off_qnorm);
  uint64_t* thr = reinterpret_cast<uint64_t*>(w + b.off_thr);
  uint32_t* count = reinterpret_cast<uint32_t*>(w + b.off_count);
  uint64_t* cand = reinterpret_cast<uint64_t*>(w + b.off_cand);
  uint64_t* cand_ub = reinterpret_cast<uint64_t*>(w + b.off_cand_ub);
  const int64_t nq_pad8 = (nq + 255) / 256 * 256;
  // (the query prep also empties thr and zeroes the counts)
  int rc = launch_qprep8(Q, nq, nq_pad8, (int)d, b.dq, metric,
                         reinterpret_cast<int8_t*>(w + b.off_qh),
                         reinterpret_cast<float*>(w + b.off_qinfo), st, thr, count);
  if (rc) return rc;
  if (metric == FX_METRIC_COS) {  // the scan's max(|q|, 1e-12) for the exact distances
    rc = launch_qnorm(Q, nq, (int)d, qnorm, st, 0);
    if (rc) return rc;
  }
  auto args = [&](int ph) {
    FilterArgs a = {};
    a.X = image;
    a.dtype = FX_DTYPE_F16;
    a.rowinfo = rowinfo;
    a.n = n;
    a.d = (int)d;
    a.row_base = row_base;
    a.Qh = reinterpret_cast<const uint16_t*>(w + b.off_qh);
    a.dq = b.dq;
    a.qstride = nq_pad8;
    a.img8 = 1;
    a.perm_a = image8_perm(n);
    a.qinfo = reinterpret_cast<const float*>(w + b.off_qinfo);
    a.nq = nq;
    a.mask = mask;
    a.tile_start = b.start[ph];
    a.tile_stride = b.stride[ph];
    a.num_tiles = b.num[ph];
    a.thr = thr;
    a.count = count;
    a.cand = cand;
    a.cap = (int)b.cap;
    a.diag = diag_env("FX_FILTER_DIAG", 0);
    return a;
  };
  // the exact k-th of the k best upper bounds in `keys` -> thr (one fused
  // launch when the buffer fits one workgroup's LDS)
  uint64_t* prune = reinterpret_cast<uint64_t*>(w + b.off_prune);
  int64_t* topr = reinterpret_cast<int64_t*>(w + b.off_topr);
  auto exact_threshold = [&](const uint64_t* keys, bool zero, const uint64_t* gate = nullptr,
                             int64_t gate_num = 0, int64_t gate_den = 1) {
    return launch_exact_threshold(X, dtype, n, (int)d, row_base, Q, qnorm, nq, keys, b.cap, count,
                                  zero, (int)k, metric, thr, st, prune, topr, gate, gate_num,
                                  gate_den);
  };
  const int m = b.nphases;
  for (int ph = 0; ph + 2 < m; ++ph) {  // sampling phases: thresholds only
    FilterArgs a = args(ph);
    a.all_pass = ph == 0 ? 1 : 0;
    a.ub_test = ph > 0 && option(kOptBatchUbTest) != 0 ? 1 : 0;
    rc = launch_filter(a, metric, st);
    if (rc) return rc;
    // (both reset the counts they read: the next phase appends from 0)
    rc = ph + 3 == m ? exact_threshold(cand, true)
                     : launch_sample_threshold(cand, nq, b.cap, count, true, (int)k, thr, st,
                                               prune);
    if (rc) return rc;
  }
  // F1: the last sample's tiles (with one phase: every tile), both bounds
  FilterArgs f1 = args(m >= 2 ? m - 2 : 0);
  f1.all_pass = m <= 2 ? 1 : 0;
  f1.cand_ub = cand_ub;
  rc = launch_filter(f1, metric, st);
  if (rc) return rc;
  if (m >= 2) {
    const int64_t t1 = b.num[m - 2], t2 = b.tiles - t1;
    // F1's threshold, then (t2 > 0) the overflow gate on it (launch_overflow_gate's
    // prediction, run by the select's own workgroups)
    rc = t2 > 0 ? exact_threshold(cand_ub, false, cand, t2, t1) : exact_threshold(cand_ub, false);
    if (rc) return rc;
    if (t2 > 0) {
      // F2: the tiles after F1's prefix
      FilterArgs f2 = args(m - 1);
      f2.tile_start = t1;
      f2.num_tiles = t2;
      f2.cand_ub = cand_ub;
      f2.skip_full = 1;
      rc = launch_filter(f2, metric, st);
      if (rc) return rc;
    }
  }
  // the final threshold only pays for itself on a batch: one or two queries
  // rescore every candidate under F1's threshold instead (a few thousand 3 KB
  // rows, ~3-6 us spread over the chip, against a ~25 us one-workgroup select)
  if (m < 2 || nq > kI8RescoreAllMaxQ) {
    rc = exact_threshold(cand_ub, false);
    if (rc) return rc;
  }
  return launch_rescore(X, dtype, n, (int)d, row_base, Q, qnorm, nq, count, cand, (int)b.cap,
                        metric, thr, st);
}

#ifdef FX_DIAG_BUILD
static int batched_phases(const BatchLayout& b, const float* X, int64_t n, int64_t d,
                          int64_t row_base, const float* Q, int64_t nq, int metric, int64_t k,
                          const uint32_t* mask, char* w, hipStream_t st) {
  float* qnorm = reinterpret_cast<float*>(w + b.off_qnorm);
  uint64_t* thr = reinterpret_cast<uint64_t*>(w + b.off_thr);
  uint32_t* count = reinterpret_cast<uint32_t*>(w + b.off_count);
  uint64_t* cand = reinterpret_cast<uint64_t*>(w + b.off_cand);
  const bool l2 = metric == FX_METRIC_L2;
  int rc = launch_qnorm(Q, nq, (int)d, qnorm, st, l2 ? 1 : 0);
  if (rc) return rc;
  // fp32 error bound of |x|^2 + |q|^2 - 2 x.q relative to |x|^2 + |q|^2:
  // 2 gamma_d for the three d-term sums + a few roundings, with 25 % slack
  const float l2_eps = (float)((2.0 * (double)d + 8.0) * 5.9604644775390625e-08 * 1.25);
  hipError_t e = hipMemsetAsync(thr, 0xFF, (size_t)nq * 8, st);
  for (int ph = 0; ph < b.nphases && e == hipSuccess; ++ph) {
    e = hipMemsetAsync(count, 0, (size_t)nq * 4 * kCountStride, st);
    if (e == hipSuccess) e = hipMemsetAsync(cand, 0xFF, (size_t)nq * b.cap * 8, st);
    if (e != hipSuccess) break;
    BatchArgs a = {};
    a.X = X;
    a.n = n;
    a.d = (int)d;
    a.row_base = row_base;
    a.Q = Q;
    a.qnorm = qnorm;
    a.nq = nq;
    a.mask = mask;
    a.tile_start = b.start[ph];
    a.tile_stride = b.stride[ph];
    a.num_tiles = b.num[ph];
    a.thr = thr;
    a.count = count;
    a.cand = cand;
    a.cap = (int)b.cap;
    a.l2_eps = l2_eps;
    rc = launch_batch(a, metric, st);
    if (rc) return rc;
    if (l2) {  // approximate keys -> exact distances before any select
      rc = launch_rescore(X, FX_DTYPE_F32, n, (int)d, row_base, Q, nullptr, nq, count, cand,
                          (int)b.cap, FX_METRIC_L2, nullptr, st);
      if (rc) return rc;
    }
    if (ph + 1 < b.nphases) {
      // the k-th composite of this sample bounds the global k-th from above
      rc = run_merge(b.merge, cand, nq, k, w + b.off_merge, nullptr, nullptr, st, thr);
      if (rc) return rc;
    }
  }
  if (e != hipSuccess) {
    set_error("batched memset: %s", hipGetErrorString(e));
    return FX_EHIP;
  }
  return FX_OK;
}
#endif  // FX_DIAG_BUILD

}  // namespace fx

using namespace fx;

extern "C" {

int fx_version(void) { return 104; }

const char* fx_last_error(void) { return g_err; }

int fx_set_option(const char* name, int64_t value) {
  const int i = option_index(name);
  if (i < 0) {
    set_error("unknown option %s", name ? name : "(null)");
    return FX_EINVAL;
  }
  if (i == kOptI8MaxK && (value < 0 || value > kSelectMaxK)) {
    set_error("option i8_max_k=%lld outside [0, %d] (the select kernel's LDS bound)",
              (long long)value, kSelectMaxK);
    return FX_EINVAL;
  }
  g_opts[i].store(value, std::memory_order_relaxed);
  return FX_OK;
}

int fx_get_option(const char* name, int64_t* out) {
  const int i = option_index(name);
  if (i < 0 || out == nullptr) {
    set_error("unknown option %s", name ? name : "(null)");
    return FX_EINVAL;
  }
  *out = g_opts[i].load(std::memory_order_relaxed);
  return FX_OK;
}

uint64_t fx_host_sync_count(void) { return g_host_syncs.load(std::memory_order_relaxed); }

int fx_device_count(int* out) {
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    set_error("hipGetDeviceCount: %s", hipGetErrorString(e));
    *out = 0;
    return FX_EHIP;
  }
  *out = c;
  return FX_OK;
}

int64_t fx_max_k(void) { return kMaxK; }

int fx_knn_workspace_bytes(int64_t n, int64_t d, int dtype, int64_t nq, int64_t k,
                           size_t* out_bytes) {
  return fx_knn_workspace_bytes_img8(n, d, dtype, nq, k, 1, out_bytes);
}

int fx_knn_workspace_bytes_img8(int64_t n, int64_t d, int dtype, int64_t nq, int64_t k,
                                int img8, size_t* out_bytes) {
  if (!out_bytes) {
    set_error("out_bytes is null");
    return FX_EINVAL;
  }
  int rc = validate(n, d, dtype, nq, 0);
  if (rc) return rc;
  if (k < 1 || k > kLargeMaxK) {
    set_error("k=%lld outside [1, %lld]", (long long)k, (long long)kLargeMaxK);
    return FX_EUNSUPPORTED;
  }
  size_t best = 0;
  for (int metric = 0; metric < 3; ++metric) {
    for (int aligned = 0; aligned < 2; ++aligned) {
      // with an int8 image a search may still plan without it (k above
      // i8_max_k): the larger of both; without one, the image-free plan only
      for (int with8 = 0; with8 < (img8 ? 2 : 1); ++with8) {
        SearchLayout s;
        rc = plan_search(n, d, dtype, nq, k, metric, aligned != 0, &s, with8 != 0);
        if (rc) return rc;
        if (s.total > best) best = s.total;
      }
    }
  }
  *out_bytes = best;
  return FX_OK;
}

static int search_layout(const void* corpus, int dtype, int64_t n, int64_t d, int64_t nq,
                         int metric, int64_t k, void* ws, size_t ws_bytes, SearchLayout* s,
                         bool img8 = false) {
  int rc = validate(n, d, dtype, nq, metric);
  if (rc) return rc;
  if (k < 1 || k > kLargeMaxK) {
    set_error("k=%lld outside [1, %lld]", (long long)k, (long long)kLargeMaxK);
    return FX_EUNSUPPORTED;
  }
  if (!corpus || !ws) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  const bool aligned = ((uintptr_t)corpus % 16) == 0;
  rc = plan_search(n, d, dtype, nq, k, metric, aligned, s, img8);
  if (rc) return rc;
  if (ws_bytes < s->total) {
    set_error("workspace too small: %zu < %zu", ws_bytes, s->total);
    return FX_EINVAL;
  }
  return FX_OK;
}

}  // extern "C"

// a filter image applies to rows of whole 16-B pieces (d % 8 == 0) through
// the filter: an fp16 image to f32 rows, an int8 image to f32 or f16 rows
static bool image_applies(const SearchLayout& s, int dtype, int64_t d, bool img8, int64_t k) {
  if (img8 && k > i8_max_k()) return false;
  return s.batched && s.batch.filter && d % 8 == 0 &&
         (dtype == FX_DTYPE_F32 || (img8 && dtype == FX_DTYPE_F16));
}

static int scan_impl(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                     const void* image, const float* rowinfo, bool img8, const float* queries,
                     int64_t nq, int metric, int64_t k, const uint32_t* mask, void* ws,
                     size_t ws_bytes, void* stream) {
  SearchLayout s;
  int rc = search_layout(corpus, dtype, n, d, nq, metric, k, ws, ws_bytes, &s,
                         img8 && image != nullptr);
  if (rc) return rc;
  if (!queries) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  if (row_base < 0 || row_base + n >= 0xffffffffll) {
    set_error("global rows [%lld, %lld) exceed the 32-bit row space", (long long)row_base,
              (long long)(row_base + n));
    return FX_EUNSUPPORTED;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (s.batched) {
    if (s.batch.filter) {
      const bool img = image != nullptr && image_applies(s, dtype, d, img8, k);
      if (img && (rowinfo == nullptr || (uintptr_t)image % 16 != 0)) {
        set_error("filter image: null row info or image not 16-byte aligned");
        return FX_EINVAL;
      }
      if (img && img8) {  // int8 image: denser samples (filter_phases)
        BatchLayout b = s.batch;
        const int64_t rmax = b.cap / (4 * k);
        const int64_t o1 = option(kOptI8SampleRatio) >= 2 ? option(kOptI8SampleRatio) : 2;
        const int64_t o2 = option(kOptI8GrowRatio) >= 2 ? option(kOptI8GrowRatio) : 2;
        int64_t r1 = rmax < o1 ? rmax : o1;
        int64_t r2 = rmax < o2 ? rmax : o2;
        const int64_t v = option(kOptBatchRatio);  // test switch: any ratio up to rmax
        if (v >= 2) r1 = r2 = v < rmax ? v : rmax;
        rc = plan_phases_i8(&b, filter_tile_rows(dtype), r1, r2);
        if (rc) return rc;
        return filter_phases_i8(b, corpus, dtype, image, rowinfo, n, d, row_base, queries, nq,
                                metric, k, mask, reinterpret_cast<char*>(ws), st);
      }
      return filter_phases(s.batch, corpus, dtype, img ? image : nullptr, rowinfo, false, n, d,
                           row_base, queries, nq, metric, k, mask, reinterpret_cast<char*>(ws),
                           st);
    }
#ifdef FX_DIAG_BUILD
    return batched_phases(s.batch, reinterpret_cast<const float*>(corpus), n, d, row_base,
                          queries, nq, metric, k, mask, reinterpret_cast<char*>(ws), st);
#endif
  }
  if (s.large) {
    ScanArgs a = {};
    a.X = corpus;
    a.n = n;
    a.d = (int)d;
    a.row_base = row_base;
    a.mask = mask;
    a.rows_per_block = s.scan.rows_per_block;
    a.cap = s.scan.cap;
    a.qbytes = s.scan.qbytes;
    a.q = queries;
    return large_scan(s.scan, a, nq, s.lg, reinterpret_cast<char*>(ws), st);
  }
  uint64_t* lists = reinterpret_cast<uint64_t*>(ws);
  ScanArgs a = {};
  a.X = corpus;
  a.n = n;
  a.d = (int)d;
  a.row_base = row_base;
  a.mask = mask;
  a.rows_per_block = s.scan.rows_per_block;
  a.k = (int)k;
  a.cap = s.scan.cap;
  a.qbytes = s.scan.qbytes;
  a.mode = kModeTopk;
  for (int64_t q0 = 0; q0 < nq; q0 += 65535) {
    const int64_t qn = (nq - q0) < 65535 ? (nq - q0) : 65535;
    a.q = queries + (size_t)q0 * d;
    a.out_lists = lists + (size_t)q0 * s.scan.nlists * k;
    rc = launch_scan(s.scan, a, qn, st);
    if (rc) return rc;
  }
  return FX_OK;
}

extern "C" {

int fx_knn_scan(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                const float* queries, int64_t nq, int metric, int64_t k,
                const uint32_t* mask, void* ws, size_t ws_bytes, void* stream) {
  return scan_impl(corpus, dtype, n, d, row_base, nullptr, nullptr, false, queries, nq, metric, k,
                   mask, ws, ws_bytes, stream);
}

int fx_knn_scan_img(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                    const void* image, const float* rowinfo, const float* queries, int64_t nq,
                    int metric, int64_t k, const uint32_t* mask, void* ws, size_t ws_bytes,
                    void* stream) {
  return scan_impl(corpus, dtype, n, d, row_base, image, rowinfo, false, queries, nq, metric, k,
                   mask, ws, ws_bytes, stream);
}

int fx_knn_scan_img8(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                     const void* image, const float* rowinfo, const float* queries, int64_t nq,
                     int metric, int64_t k, const uint32_t* mask, void* ws, size_t ws_bytes,
                     void* stream) {
  return scan_impl(corpus, dtype, n, d, row_base, image, rowinfo, true, queries, nq, metric, k,
                   mask, ws, ws_bytes, stream);
}

int fx_filter_image_bytes(int64_t n, int64_t d, size_t* image_bytes, size_t* rowinfo_bytes) {
  if (!image_bytes || !rowinfo_bytes) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  if (n < 0 || d < 8 || d % 8 != 0) {
    set_error("filter image: n=%lld d=%lld (d must be a positive multiple of 8)", (long long)n,
              (long long)d);
    return FX_EUNSUPPORTED;
  }
  *image_bytes = image_tiled() ? (size_t)((n + 31) / 32) * (size_t)((d + 15) / 16) * 1024
                               : (size_t)n * (size_t)d * 2;
  *rowinfo_bytes = (size_t)n * 4;
  return FX_OK;
}

int fx_filter_image(const float* corpus, int64_t n, int64_t d, void* image, float* rowinfo,
                    void* stream) {
  size_t ib = 0, rb = 0;
  int rc = fx_filter_image_bytes(n, d, &ib, &rb);
  if (rc) return rc;
  if (n > 0 && (!corpus || !image || !rowinfo)) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  if ((uintptr_t)corpus % 16 != 0 || (uintptr_t)image % 16 != 0) {
    set_error("filter image: corpus and image must be 16-byte aligned");
    return FX_EINVAL;
  }
  if (d > 0x7fffffffll) {
    set_error("filter image: d=%lld too large", (long long)d);
    return FX_EUNSUPPORTED;
  }
  return launch_image(corpus, n, (int)d, image, rowinfo, reinterpret_cast<hipStream_t>(stream));
}

int fx_filter_image8_bytes(int64_t n, int64_t d, size_t* image_bytes, size_t* rowinfo_bytes) {
  if (!image_bytes || !rowinfo_bytes) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  if (n < 0 || d < 8 || d % 8 != 0) {
    set_error("filter image: n=%lld d=%lld (d must be a positive multiple of 8)", (long long)n,
              (long long)d);
    return FX_EUNSUPPORTED;
  }
  *image_bytes = (size_t)((n + 31) / 32) * (size_t)((d + 31) / 32) * 1024;
  *rowinfo_bytes = (size_t)n * kI8RowInfo * 4;
  return FX_OK;
}

int fx_filter_image8_perm(int64_t n, uint64_t* mult) {
  if (!mult || n < 0) {
    set_error("fx_filter_image8_perm: n=%lld", (long long)n);
    return FX_EINVAL;
  }
  *mult = image8_perm(n);
  return FX_OK;
}

int fx_filter_image8(const float* corpus, int64_t n, int64_t d, void* image, float* rowinfo,
                     void* stream) {
  return fx_filter_image8_typed(corpus, FX_DTYPE_F32, n, d, image, rowinfo, stream);
}

int fx_filter_image8_typed(const void* corpus, int dtype, int64_t n, int64_t d, void* image,
                           float* rowinfo, void* stream) {
  if (dtype != FX_DTYPE_F32 && dtype != FX_DTYPE_F16) {
    set_error("filter image: dtype %d is not float32 or float16", dtype);
    return FX_EINVAL;
  }
  size_t ib = 0, rb = 0;
  int rc = fx_filter_image8_bytes(n, d, &ib, &rb);
  if (rc) return rc;
  if (n > 0 && (!corpus || !image || !rowinfo)) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  if ((uintptr_t)corpus % 16 != 0 || (uintptr_t)image % 16 != 0 || (uintptr_t)rowinfo % 16 != 0) {
    set_error("filter image: corpus, image and row info must be 16-byte aligned");
    return FX_EINVAL;
  }
  if (d > 0x7fffffffll) {
    set_error("filter image: d=%lld too large", (long long)d);
    return FX_EUNSUPPORTED;
  }
  return launch_image8(corpus, dtype, n, (int)d, image, rowinfo,
                       reinterpret_cast<hipStream_t>(stream));
}

int fx_filter_image_used(int64_t n, int64_t d, int dtype, int64_t nq, int64_t k, int metric,
                         int* out) {
  if (!out) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  *out = 0;
  int rc = validate(n, d, dtype, nq, metric);
  if (rc) return rc;
  if (k < 1 || k > kLargeMaxK) {
    set_error("k=%lld outside [1, %lld]", (long long)k, (long long)kLargeMaxK);
    return FX_EUNSUPPORTED;
  }
  SearchLayout s;
  // (the int8 image, the host's default, also serves single queries over
  // large corpora: use_batched)
  const bool img8 = option(kOptFilterImage) == 8;
  rc = plan_search(n, d, dtype, nq, k, metric, true, &s, img8);
  if (rc) return rc;
  *out = image_applies(s, dtype, d, img8, k) ? 1 : 0;
  return FX_OK;
}

static int reduce_impl(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                       const float* queries, int64_t nq, int metric, int64_t k,
                       const uint32_t* mask, void* ws, size_t ws_bytes, float* out_dist,
                       int64_t* out_row, void* stream, bool img8) {
  SearchLayout s;
  int rc = search_layout(corpus, dtype, n, d, nq, metric, k, ws, ws_bytes, &s, img8);
  if (rc) return rc;
  if (!out_dist || !out_row) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (s.large) {
    return large_reduce(n, nq, k, s.lg, reinterpret_cast<char*>(ws), out_dist, out_row, st);
  }
  if (!s.batched) {
    const uint64_t* lists = reinterpret_cast<const uint64_t*>(ws);
    void* mws = reinterpret_cast<char*>(ws) + s.lists_bytes;
    return run_merge(s.merge, lists, nq, k, mws, out_dist, out_row, st);
  }
  // batched: final select over the last phase's candidates
  const BatchLayout& b = s.batch;
  char* w = reinterpret_cast<char*>(ws);
  const uint64_t* cand = reinterpret_cast<const uint64_t*>(w + b.off_cand);
  uint32_t* count = reinterpret_cast<uint32_t*>(w + b.off_count);
  // queries whose candidates overflowed `cap` are recomputed exactly, gated
  // on the device ("force_fallback" (test switch): every query)
  const int64_t gate_cap = option(kOptForceFallback) != 0 ? -1 : b.cap;
  if (b.img8 && s.fb_queries >= nq) {
    // one round: the gated scan's lists feed the final select of the
    // overflowing queries (no merge levels of their own)
    const uint64_t* lists = nullptr;
    rc = fallback_scan(s, corpus, n, d, row_base, queries, nq, k, mask, count, gate_cap,
                       w + s.single_off, st, &lists);
    if (rc) return rc;
    return launch_final_select(cand, nq, b.cap, count, (int)k, out_dist, out_row, lists,
                               s.scan.nlists * k, gate_cap, st,
                               reinterpret_cast<uint64_t*>(w + b.off_prune));
  }
  // (the fallback gate reads the counts next: kept)
  rc = b.img8 ? launch_final_select(cand, nq, b.cap, count, (int)k, out_dist, out_row, nullptr, 0,
                                    0, st, reinterpret_cast<uint64_t*>(w + b.off_prune))
              : run_merge(b.merge, cand, nq, k, w + b.off_merge, out_dist, out_row, st, nullptr,
                          nullptr, 0, count);
  if (rc) return rc;
  return fallback_search(s, corpus, dtype, n, d, row_base, queries, nq, metric, k, mask, count,
                         gate_cap, w + s.single_off, out_dist, out_row, st);
}

int fx_knn_filter_state(const void* corpus, int dtype, int64_t n, int64_t d, int64_t nq,
                        int metric, int64_t k, int img8, const void* ws, size_t ws_bytes,
                        uint64_t* out_thr, uint64_t* out_cand, uint64_t* out_cand_ub,
                        void* stream) {
  SearchLayout s;
  int rc = search_layout(corpus, dtype, n, d, nq, metric, k, const_cast<void*>(ws), ws_bytes, &s,
                         img8 != 0);
  if (rc) return rc;
  if (!s.batched || !s.batch.filter) {
    set_error("fx_knn_filter_state: the search did not run the filter");
    return FX_EINVAL;
  }
  const char* w = reinterpret_cast<const char*>(ws);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const size_t cb = (size_t)nq * s.batch.cap * 8;
  hipError_t e = hipSuccess;
  if (out_thr) e = hipMemcpyAsync(out_thr, w + s.batch.off_thr, (size_t)nq * 8,
                                  hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess && out_cand)
    e = hipMemcpyAsync(out_cand, w + s.batch.off_cand, cb, hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess && out_cand_ub)
    e = hipMemcpyAsync(out_cand_ub, w + s.batch.off_cand_ub, cb, hipMemcpyDeviceToDevice, st);
  if (e != hipSuccess) {
    set_error("fx_knn_filter_state: %s", hipGetErrorString(e));
    return FX_EHIP;
  }
  return FX_OK;
}

int fx_knn_filter_counts(const void* corpus, int dtype, int64_t n, int64_t d, int64_t nq,
                         int metric, int64_t k, int img8, const void* ws, size_t ws_bytes,
                         uint32_t* out_counts, int64_t* out_cap, void* stream) {
  SearchLayout s;
  int rc = search_layout(corpus, dtype, n, d, nq, metric, k, const_cast<void*>(ws), ws_bytes, &s,
                         img8 != 0);
  if (rc) return rc;
  if (!out_counts || !out_cap) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  if (!s.batched) {
    *out_cap = -1;
    return FX_OK;
  }
  *out_cap = s.batch.cap;
  const char* c = reinterpret_cast<const char*>(ws) + s.batch.off_count;
  hipError_t e = hipMemcpy2DAsync(out_counts, 4, c, 4 * kCountStride, 4, (size_t)nq,
                                  hipMemcpyDeviceToDevice, reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) {
    set_error("fx_knn_filter_counts: %s", hipGetErrorString(e));
    return FX_EHIP;
  }
  return FX_OK;
}

int fx_knn_reduce(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                  const float* queries, int64_t nq, int metric, int64_t k,
                  const uint32_t* mask, void* ws, size_t ws_bytes, float* out_dist,
                  int64_t* out_row, void* stream) {
  return reduce_impl(corpus, dtype, n, d, row_base, queries, nq, metric, k, mask, ws, ws_bytes,
                     out_dist, out_row, stream, false);
}

int fx_knn_reduce_img8(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                       const void* image, const float* queries, int64_t nq, int metric, int64_t k,
                       const uint32_t* mask, void* ws, size_t ws_bytes, float* out_dist,
                       int64_t* out_row, void* stream) {
  return reduce_impl(corpus, dtype, n, d, row_base, queries, nq, metric, k, mask, ws, ws_bytes,
                     out_dist, out_row, stream, image != nullptr);
}

int fx_knn_search(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                  const float* queries, int64_t nq, int metric, int64_t k,
                  const uint32_t* mask, void* ws, size_t ws_bytes, float* out_dist,
                  int64_t* out_row, void* stream) {
  if (!out_dist || !out_row) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  int rc = fx_knn_scan(corpus, dtype, n, d, row_base, queries, nq, metric, k, mask, ws, ws_bytes,
                       stream);
  if (rc) return rc;
  return fx_knn_reduce(corpus, dtype, n, d, row_base, queries, nq, metric, k, mask, ws, ws_bytes,
                       out_dist, out_row, stream);
}

int fx_knn_search_img(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                      const void* image, const float* rowinfo, const float* queries, int64_t nq,
                      int metric, int64_t k, const uint32_t* mask, void* ws, size_t ws_bytes,
                      float* out_dist, int64_t* out_row, void* stream) {
  if (!out_dist || !out_row) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  int rc = fx_knn_scan_img(corpus, dtype, n, d, row_base, image, rowinfo, queries, nq, metric, k,
                           mask, ws, ws_bytes, stream);
  if (rc) return rc;
  return fx_knn_reduce(corpus, dtype, n, d, row_base, queries, nq, metric, k, mask, ws, ws_bytes,
                       out_dist, out_row, stream);
}

int fx_knn_search_img8(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                       const void* image, const float* rowinfo, const float* queries, int64_t nq,
                       int metric, int64_t k, const uint32_t* mask, void* ws, size_t ws_bytes,
                       float* out_dist, int64_t* out_row, void* stream) {
  if (!out_dist || !out_row) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  int rc = fx_knn_scan_img8(corpus, dtype, n, d, row_base, image, rowinfo, queries, nq, metric, k,
                            mask, ws, ws_bytes, stream);
  if (rc) return rc;
  return reduce_impl(corpus, dtype, n, d, row_base, queries, nq, metric, k, mask, ws, ws_bytes,
                     out_dist, out_row, stream, image != nullptr);
}

int fx_knn_search_rows_workspace_bytes(int64_t nrows, int64_t d, int dtype, int64_t nq,
                                       int64_t k, size_t* out_bytes) {
  if (!out_bytes) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  int rc = validate(nrows, d, dtype, nq, FX_METRIC_L2);
  if (rc) return rc;
  if (k < 1 || k > kLargeMaxK) {
    set_error("k=%lld outside [1, %lld]", (long long)k, (long long)kLargeMaxK);
    return FX_EUNSUPPORTED;
  }
  SearchLayout s;
  rc = k > kMaxK ? plan_large_search(nrows, d, dtype, nq, FX_METRIC_L2, true, &s)
                 : plan_single(nrows, d, dtype, nq, k, FX_METRIC_L2, true, &s);
  if (rc) return rc;
  *out_bytes = s.total;
  return FX_OK;
}

int fx_knn_search_rows(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                       const int32_t* rows, int64_t nrows, const float* queries, int64_t nq,
                       int metric, int64_t k, void* ws, size_t ws_bytes, float* out_dist,
                       int64_t* out_row, void* stream) {
  int rc = validate(nrows, d, dtype, nq, metric);
  if (rc) return rc;
  if (k < 1 || k > kLargeMaxK) {
    set_error("k=%lld outside [1, %lld]", (long long)k, (long long)kLargeMaxK);
    return FX_EUNSUPPORTED;
  }
  if (!corpus || !ws || !queries || !out_dist || !out_row || (nrows > 0 && !rows)) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  if (row_base < 0 || n < 0 || row_base + n >= 0xffffffffll || n > 0x7fffffffll) {
    set_error("global rows [%lld, %lld) exceed the 32-bit row space", (long long)row_base,
              (long long)(row_base + n));
    return FX_EUNSUPPORTED;
  }
  SearchLayout s;
  const bool aligned = ((uintptr_t)corpus % 16) == 0;
  rc = k > kMaxK ? plan_large_search(nrows, d, dtype, nq, metric, aligned, &s)
                 : plan_single(nrows, d, dtype, nq, k, metric, aligned, &s);
  if (rc) return rc;
  if (ws_bytes < s.total) {
    set_error("workspace too small: %zu < %zu", ws_bytes, s.total);
    return FX_EINVAL;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (s.large) {
    ScanArgs a = {};
    a.X = corpus;
    a.n = nrows;
    a.d = (int)d;
    a.row_base = row_base;
    a.rows = rows;
    a.rows_per_block = s.scan.rows_per_block;
    a.cap = s.scan.cap;
    a.qbytes = s.scan.qbytes;
    a.q = queries;
    rc = large_scan(s.scan, a, nq, s.lg, reinterpret_cast<char*>(ws), st);
    if (rc) return rc;
    return large_reduce(nrows, nq, k, s.lg, reinterpret_cast<char*>(ws), out_dist, out_row, st);
  }
  uint64_t* lists = reinterpret_cast<uint64_t*>(ws);
  ScanArgs a = {};
  a.X = corpus;
  a.n = nrows;
  a.d = (int)d;
  a.row_base = row_base;
  a.rows = rows;
  a.rows_per_block = s.scan.rows_per_block;
  a.k = (int)k;
  a.cap = s.scan.cap;
  a.qbytes = s.scan.qbytes;
  a.mode = kModeTopk;
  for (int64_t q0 = 0; q0 < nq; q0 += 65535) {
    const int64_t qn = (nq - q0) < 65535 ? (nq - q0) : 65535;
    a.q = queries + (size_t)q0 * d;
    a.out_lists = lists + (size_t)q0 * s.scan.nlists * k;
    rc = launch_scan(s.scan, a, qn, st);
    if (rc) return rc;
  }
  return run_merge(s.merge, lists, nq, k, reinterpret_cast<char*>(ws) + s.lists_bytes, out_dist,
                   out_row, st);
}

int fx_knn_distances(const void* corpus, int dtype, int64_t n, int64_t d,
                     const float* queries, int64_t nq, int metric, const uint32_t* mask,
                     float* out, void* stream) {
  int rc = validate(n, d, dtype, nq, metric);
  if (rc) return rc;
  if (!corpus || !queries || !out) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  const bool aligned = ((uintptr_t)corpus % 16) == 0;
  ScanPlan p;
  rc = plan_scan(n, d, dtype, 1, metric, aligned, &p);
  if (rc) return rc;
  ScanArgs a = {};
  a.X = corpus;
  a.n = n;
  a.d = (int)d;
  a.row_base = 0;
  a.mask = mask;
  a.rows_per_block = p.rows_per_block;
  a.k = 1;
  a.cap = p.cap;
  a.qbytes = p.qbytes;
  a.mode = kModeDist;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int64_t q0 = 0; q0 < nq; q0 += 65535) {
    const int64_t qn = (nq - q0) < 65535 ? (nq - q0) : 65535;
    a.q = queries + (size_t)q0 * d;
    a.out_dist = out + (size_t)q0 * n;
    rc = launch_scan(p, a, qn, st);
    if (rc) return rc;
  }
  return FX_OK;
}

// merges of lists longer than the fused path's k go through the radix sort
static bool merge_is_large(int64_t kin, int64_t k) { return k > kMaxK || kin > kMaxK; }

int fx_topk_merge_workspace_bytes(int64_t nq, int64_t parts, int64_t kin, int64_t k,
                                  size_t* out_bytes) {
  if (!out_bytes || nq < 1 || parts < 1 || kin < 1 || k < 1 || k > kLargeMaxK ||
      parts * kin > kLargeMaxK) {
    set_error("invalid merge shape");
    return FX_EINVAL;
  }
  if (merge_is_large(kin, k)) {
    *out_bytes = plan_large(parts * kin, nq).total;
    return FX_OK;
  }
  MergePlan mp;
  int rc = plan_merge(nq, parts, kin, k, &mp);
  if (rc) return rc;
  *out_bytes = align256((size_t)nq * parts * kin * 8) + mp.ws_bytes;
  return FX_OK;
}

int fx_topk_merge(const float* in_dist, const int64_t* in_row, int64_t nq, int64_t parts,
                  int64_t kin, int64_t k, void* ws, size_t ws_bytes, float* out_dist,
                  int64_t* out_row, void* stream) {
  size_t need = 0;
  int rc = fx_topk_merge_workspace_bytes(nq, parts, kin, k, &need);
  if (rc) return rc;
  if (!in_dist || !in_row || !ws || !out_dist || !out_row) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  if (ws_bytes < need) {
    set_error("workspace too small: %zu < %zu", ws_bytes, need);
    return FX_EINVAL;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (merge_is_large(kin, k)) {
    const LargeLayout l = plan_large(parts * kin, nq);
    char* w = reinterpret_cast<char*>(ws);
    rc = launch_encode(in_dist, in_row, nq * parts * kin,
                       reinterpret_cast<uint64_t*>(w + l.off_keys), st);
    if (rc) return rc;
    return large_reduce(parts * kin, nq, k, l, w, out_dist, out_row, st);
  }
  MergePlan mp;
  rc = plan_merge(nq, parts, kin, k, &mp);
  if (rc) return rc;
  uint64_t* comp = reinterpret_cast<uint64_t*>(ws);
  void* mws = reinterpret_cast<char*>(ws) + align256((size_t)nq * parts * kin * 8);
  rc = launch_encode(in_dist, in_row, nq * parts * kin, comp, st);
  if (rc) return rc;
  return run_merge(mp, comp, nq, k, mws, out_dist, out_row, st);
}

int fx_fill_normal(void* x, int dtype, int64_t n, int64_t d, uint64_t seed, int64_t row_base,
                   int64_t cluster, void* stream) {
  if (!x || n < 0 || d < 1 || (dtype != FX_DTYPE_F32 && dtype != FX_DTYPE_F16)) {
    set_error("invalid fill arguments");
    return FX_EINVAL;
  }
  return launch_fill(x, dtype, n, d, seed, row_base, cluster,
                     reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"
