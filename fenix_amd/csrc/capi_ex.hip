// Corpus-descriptor entry points (include/fenix_knn.h fx_corpus): every
// dtype including FX_DTYPE_QU8 (quint8 codes dequantised in the scan's
// registers, ex/arrow/quint8/quint8.py:81-84), optional row list and mask.
// Same plans and kernels as fx_knn_search / fx_knn_search_rows /
// fx_knn_distances; no batched MFMA path here (it reads f32 rows).
#include <vector>

#include "fx_internal.h"

namespace fx {
namespace {

constexpr int64_t kMaxKEx = 1024;  // fused path; larger k: knn_large.hip

size_t align256(size_t v) { return (v + 255) / 256 * 256; }

int check_corpus(const fx_corpus* c, int64_t nq, int metric) {
  if (c == nullptr || c->data == nullptr) {
    set_error("null corpus");
    return FX_EINVAL;
  }
  if (c->n < 1 || c->d < 1 || nq < 1) {
    set_error("invalid shape n=%lld d=%lld nq=%lld", (long long)c->n, (long long)c->d,
              (long long)nq);
    return FX_EINVAL;
  }
  if (c->d > (1 << 20)) {
    set_error("d=%lld too large", (long long)c->d);
    return FX_EUNSUPPORTED;
  }
  if (c->dtype != FX_DTYPE_F32 && c->dtype != FX_DTYPE_F16 && c->dtype != FX_DTYPE_QU8) {
    set_error("unsupported dtype %d", c->dtype);
    return FX_EINVAL;
  }
  if (metric < FX_METRIC_L2 || metric > FX_METRIC_COS) {
    set_error("unsupported metric %d", metric);
    return FX_EINVAL;
  }
  if (c->dtype == FX_DTYPE_QU8 && (c->zero_point < 0 || c->zero_point > 255 ||
                                   !(c->scale > 0.f) || c->scale == __builtin_inff())) {
    set_error("quint8 zero_point %d / scale %g out of range", c->zero_point, (double)c->scale);
    return FX_EINVAL;
  }
  if (c->row_base < 0 || c->row_base + c->n >= 0xffffffffll || c->n > 0x7fffffffll) {
    set_error("global rows [%lld, %lld) exceed the 32-bit row space", (long long)c->row_base,
              (long long)(c->row_base + c->n));
    return FX_EUNSUPPORTED;
  }
  return FX_OK;
}

struct ExPlan {
  ScanPlan scan;
  MergePlan merge;
  size_t lists_bytes, total;
  bool large = false;
  LargeLayout lg;
};

int plan_ex(const fx_corpus* c, int64_t rows, int64_t nq, int64_t k, int metric, ExPlan* p) {
  if (k < 1 || k > 0x7fffffffll) {
    set_error("k=%lld out of range", (long long)k);
    return FX_EUNSUPPORTED;
  }
  const bool aligned = ((uintptr_t)c->data % 16) == 0;
  if (k > kMaxKEx) {
    int rc = plan_scan(rows, c->d, c->dtype, 1, metric, aligned, &p->scan);
    if (rc) return rc;
    p->large = true;
    p->lg = plan_large(rows, nq);
    p->total = p->lg.total;
    return FX_OK;
  }
  int rc = plan_scan(rows, c->d, c->dtype, k, metric, aligned, &p->scan);
  if (rc) return rc;
  rc = plan_merge(nq, p->scan.nlists, k, k, &p->merge);
  if (rc) return rc;
  p->lists_bytes = align256((size_t)nq * p->scan.nlists * k * 8);
  p->total = p->lists_bytes + p->merge.ws_bytes;
  return FX_OK;
}

ScanArgs base_args(const fx_corpus* c, const ScanPlan& p) {
  ScanArgs a = {};
  a.X = c->data;
  a.d = (int)c->d;
  a.row_base = c->row_base;
  a.rows_per_block = p.rows_per_block;
  a.cap = p.cap;
  a.qbytes = p.qbytes;
  a.qscale = c->dtype == FX_DTYPE_QU8 ? c->scale : 1.f;
  a.qshift = c->dtype == FX_DTYPE_QU8 ? (float)c->zero_point : 0.f;
  return a;
}

// fx_knn_search_shards: every shard's scan plan, and where its lists start
// in the one list buffer [nq][lists][k] the merge reads
constexpr int kMaxShards = 4096;

struct ShardsPlan {
  std::vector<ScanPlan> scan;
  std::vector<int64_t> base;
  int64_t lists = 0;
  MergePlan merge;
  size_t lists_bytes = 0, total = 0;
};

int check_shards(const fx_corpus* s, int ns, int64_t nq, int64_t k, int metric) {
  if (s == nullptr || ns < 1 || ns > kMaxShards) {
    set_error("fx_knn_search_shards: %d shards (1 .. %d)", ns, kMaxShards);
    return FX_EINVAL;
  }
  if (k < 1 || k > kMaxKEx) {
    set_error("fx_knn_search_shards: k=%lld outside [1, %lld]", (long long)k, (long long)kMaxKEx);
    return FX_EUNSUPPORTED;
  }
  for (int i = 0; i < ns; ++i) {
    int rc = check_corpus(&s[i], nq, metric);
    if (rc) return rc;
    if (s[i].d != s[0].d || s[i].dtype != s[0].dtype) {
      set_error("fx_knn_search_shards: shard %d has d=%lld dtype %d, shard 0 d=%lld dtype %d", i,
                (long long)s[i].d, s[i].dtype, (long long)s[0].d, s[0].dtype);
      return FX_EINVAL;
    }
  }
  return FX_OK;
}

int plan_shards(const fx_corpus* s, int ns, int64_t nq, int64_t k, int metric, ShardsPlan* p) {
  p->scan.resize(ns);
  p->base.resize(ns);
  p->lists = 0;
  for (int i = 0; i < ns; ++i) {
    const bool aligned = ((uintptr_t)s[i].data % 16) == 0;
    int rc = plan_scan(s[i].n, s[i].d, s[i].dtype, k, metric, aligned, &p->scan[i]);
    if (rc) return rc;
    p->base[i] = p->lists;
    p->lists += p->scan[i].nlists;
  }
  int rc = plan_merge(nq, p->lists, k, k, &p->merge);
  if (rc) return rc;
  p->lists_bytes = align256((size_t)nq * p->lists * k * 8);
  p->total = p->lists_bytes + p->merge.ws_bytes;
  return FX_OK;
}

}  // namespace
}  // namespace fx

using namespace fx;

extern "C" {

int fx_knn_search_ex_workspace_bytes(const fx_corpus* c, int64_t nrows, int64_t nq, int64_t k,
                                     size_t* out_bytes) {
  int rc = check_corpus(c, nq, FX_METRIC_L2);
  if (rc) return rc;
  if (out_bytes == nullptr) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  const int64_t rows = nrows >= 0 ? nrows : c->n;
  if (rows < 1) {
    set_error("empty row list");
    return FX_EINVAL;
  }
  ExPlan p;
  rc = plan_ex(c, rows, nq, k, FX_METRIC_L2, &p);
  if (rc) return rc;
  *out_bytes = p.total;
  return FX_OK;
}

int fx_knn_search_ex(const fx_corpus* c, const int32_t* rows, int64_t nrows,
                     const float* queries, int64_t nq, int metric, int64_t k,
                     const uint32_t* mask, void* ws, size_t ws_bytes, float* out_dist,
                     int64_t* out_row, void* stream) {
  int rc = check_corpus(c, nq, metric);
  if (rc) return rc;
  if (!queries || !ws || !out_dist || !out_row) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  const int64_t n = rows != nullptr ? nrows : c->n;
  if (n < 1) {
    set_error("empty row list");
    return FX_EINVAL;
  }
  ExPlan p;
  rc = plan_ex(c, n, nq, k, metric, &p);
  if (rc) return rc;
  if (ws_bytes < p.total) {
    set_error("workspace too small: %zu < %zu", ws_bytes, p.total);
    return FX_EINVAL;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (p.large) {
    ScanArgs a = base_args(c, p.scan);
    a.n = n;
    a.rows = rows;
    a.mask = mask;
    a.q = queries;
    rc = large_scan(p.scan, a, nq, p.lg, reinterpret_cast<char*>(ws), st);
    if (rc) return rc;
    return large_reduce(n, nq, k, p.lg, reinterpret_cast<char*>(ws), out_dist, out_row, st);
  }
  uint64_t* lists = reinterpret_cast<uint64_t*>(ws);
  ScanArgs a = base_args(c, p.scan);
  a.n = n;
  a.rows = rows;
  a.mask = mask;
  a.k = (int)k;
  a.mode = kModeTopk;
  for (int64_t q0 = 0; q0 < nq; q0 += 65535) {
    const int64_t qn = (nq - q0) < 65535 ? (nq - q0) : 65535;
    a.q = queries + (size_t)q0 * c->d;
    a.out_lists = lists + (size_t)q0 * p.scan.nlists * k;
    rc = launch_scan(p.scan, a, qn, st);
    if (rc) return rc;
  }
  return run_merge(p.merge, lists, nq, k, reinterpret_cast<char*>(ws) + p.lists_bytes, out_dist,
                   out_row, st);
}

int fx_knn_distances_ex(const fx_corpus* c, const float* queries, int64_t nq, int metric,
                        const uint32_t* mask, float* out, void* stream) {
  int rc = check_corpus(c, nq, metric);
  if (rc) return rc;
  if (!queries || !out) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  ScanPlan p;
  rc = plan_scan(c->n, c->d, c->dtype, 1, metric, ((uintptr_t)c->data % 16) == 0, &p);
  if (rc) return rc;
  ScanArgs a = base_args(c, p);
  a.n = c->n;
  a.row_base = 0;
  a.mask = mask;
  a.k = 1;
  a.mode = kModeDist;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  for (int64_t q0 = 0; q0 < nq; q0 += 65535) {
    const int64_t qn = (nq - q0) < 65535 ? (nq - q0) : 65535;
    a.q = queries + (size_t)q0 * c->d;
    a.out_dist = out + (size_t)q0 * c->n;
    rc = launch_scan(p, a, qn, st);
    if (rc) return rc;
  }
  return FX_OK;
}

int fx_knn_search_shards_workspace_bytes(const fx_corpus* shards, int nshards, int64_t nq,
                                         int64_t k, size_t* out_bytes) {
  if (out_bytes == nullptr) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  int rc = check_shards(shards, nshards, nq, k, FX_METRIC_L2);
  if (rc) return rc;
  size_t best = 0;
  for (int metric = FX_METRIC_L2; metric <= FX_METRIC_COS; ++metric) {  // (plans are per metric)
    ShardsPlan p;
    rc = plan_shards(shards, nshards, nq, k, metric, &p);
    if (rc) return rc;
    if (p.total > best) best = p.total;
  }
  *out_bytes = best;
  return FX_OK;
}

int fx_knn_search_shards(const fx_corpus* shards, int nshards, const float* queries, int64_t nq,
                         int metric, int64_t k, const uint32_t* const* masks, void* ws,
                         size_t ws_bytes, float* out_dist, int64_t* out_row, void* stream) {
  int rc = check_shards(shards, nshards, nq, k, metric);
  if (rc) return rc;
  if (!queries || !ws || !out_dist || !out_row) {
    set_error("null pointer argument");
    return FX_EINVAL;
  }
  ShardsPlan p;
  rc = plan_shards(shards, nshards, nq, k, metric, &p);
  if (rc) return rc;
  if (ws_bytes < p.total) {
    set_error("workspace too small: %zu < %zu", ws_bytes, p.total);
    return FX_EINVAL;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  uint64_t* lists = reinterpret_cast<uint64_t*>(ws);
  const int64_t d = shards[0].d;
  for (int i = 0; i < nshards; ++i) {
    ScanArgs a = base_args(&shards[i], p.scan[i]);
    a.n = shards[i].n;
    a.mask = masks != nullptr ? masks[i] : nullptr;
    a.k = (int)k;
    a.mode = kModeTopk;
    a.list_stride = p.lists;
    a.list_base = p.base[i];
    for (int64_t q0 = 0; q0 < nq; q0 += 65535) {
      const int64_t qn = (nq - q0) < 65535 ? (nq - q0) : 65535;
      a.q = queries + (size_t)q0 * d;
      a.out_lists = lists + (size_t)q0 * p.lists * k;
      rc = launch_scan(p.scan[i], a, qn, st);
      if (rc) return rc;
    }
  }
  return run_merge(p.merge, lists, nq, k, reinterpret_cast<char*>(ws) + p.lists_bytes, out_dist,
                   out_row, st);
}

}  // extern "C"
