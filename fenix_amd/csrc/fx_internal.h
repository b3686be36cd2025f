// Internal declarations shared by the kernel translation units and the C ABI.
#pragma once

#include "../../include/fenix_knn.h"
#include "fx_common.h"

namespace fx {

constexpr int kModeTopk = 0;
constexpr int kModeDist = 1;
// Per-query append counters of the batched kernels sit 128 B apart: every
// counter in its own cache line, so the L2 channels serialise fewer atomics.
constexpr int kCountStride = 32;
// largest k of the one-workgroup select_kernel (knn_batch.hip): its LDS holds a
// 16 384-entry chunk plus the k kept so far rounded up to a power of two, which
// fits the 160 KB of a CU up to 2 048; also the bound of option "i8_max_k"
constexpr int kSelectMaxK = 2048;

// Process-wide options (fx_set_option, include/fenix_knn.h); relaxed atomics.
enum Option : int {
  kOptBatched,
  kOptBatchMinQ,
  kOptBatchCap,
  kOptBatchRatio,
  kOptForceFallback,
  kOptScanInterleave,
  kOptQ8Dma,
  kOptFilterImage,  // filter image bits for f32 corpora (engine policy): 8, 16 or 0 (none)
  kOptBatchUbTest,  // sampling phases append by upper bound (0: by lower bound, test switch)
  kOptSingleImage,  // single queries over large f32 corpora through a supplied int8 image
  kOptI8MaxK,       // largest k an int8 filter image serves
  kOptImg6,         // int8 images: resident-query-slice kernel (1: <= 128 queries, 2: all, 0: off)
  kOptImg8,         // int8 images: queries-in-registers kernel for > 128 queries, d <= 768 (0: off)
  kOptI8SampleRatio,  // int8 images: F1 holds every r1-th tile (filter_phases_i8)
  kOptI8GrowRatio,    // int8 images: the samples before F1 shrink by r2 each
  kOptSelectPrune,    // int8 images: 1: selects at k >= 512 prune first; 2: any k; 0: never
  kOptCount
};
int64_t option(Option o);

// Diagnostic builds for tools/ (make diag: -DFX_DIAG_BUILD) read a few
// variant and tuning switches from the environment; the product library
// compiles the rejected variants out and takes the defaults.
#ifdef FX_DIAG_BUILD
int diag_env(const char* name, int dflt);
#else
constexpr int diag_env(const char*, int dflt) { return dflt; }
#endif

struct ScanArgs {
  const void* X;          // [n][d] corpus shard
  int64_t n;
  int d;
  int64_t row_base;       // global row of local row 0
  const float* q;         // [nq][d]
  const uint32_t* mask;   // bitmap or null
  const int32_t* rows;    // [n] corpus rows to scan (n = list length) or null: rows 0..n-1
  int64_t rows_per_block;
  int k;
  int cap;                // per-wave candidate list capacity
  size_t qbytes;          // LDS bytes reserved for the query
  int mode;               // kModeTopk / kModeDist
  uint64_t* out_lists;    // topk: [nq][list_stride][k] composites (one list per block,
                          // block b at list list_base + b)
  int64_t list_stride;    // lists per query in out_lists (0: gridDim.x)
  int64_t list_base;      // this launch's first list (fx_knn_search_shards: the shard's)
  float* out_dist;        // dist: [nq][n]
  float qscale, qshift;   // FX_DTYPE_QU8: value = qscale * (code - qshift)
  // bit 0 clear: block b scans rows [b * rows_per_block, ...) in order; set:
  // block steps of 16U rows dealt round-robin over the grid.  Bit 1: no
  // software pipeline (one tile per wave in flight).  Set by launch_scan.
  int interleave;
  // Device-side gate (the batched path's overflow fallback): when non-null, a
  // workgroup of query qi returns at once unless gate[qi * kCountStride] >
  // gate_cap (gate_cap < 0: every query runs).
  const uint32_t* gate;
  int64_t gate_cap;
};

typedef void (*ScanKernelFn)(ScanArgs);

struct ScanPlan {
  ScanKernelFn fn;
  int W, L, U, cap;
  size_t qbytes, smem;
  int64_t blocks, rows_per_block, nlists;
  int interleave;  // ScanArgs::interleave for the register-tile kernels
  // quint8 rows staged by LDS-DMA (plain contiguous scans: no mask, no row
  // list); null when not applicable.  Same rows_per_block (its U divides it).
  ScanKernelFn fn_dma;
  size_t smem_dma;
};

int plan_scan(int64_t n, int64_t d, int dtype, int64_t k, int metric, bool aligned, ScanPlan* p);
// at most max_blocks blocks per query (rows_per_block, blocks, nlists recomputed)
void limit_scan_blocks(ScanPlan* p, int64_t n, int64_t max_blocks);
int launch_scan(const ScanPlan& p, const ScanArgs& a, int64_t nq, hipStream_t stream);

// Merge of candidate lists: [nq][nlists][kin] composites -> top-k.
struct MergePlan {
  int levels;
  int64_t group[16];      // lists per block at each level
  int64_t lists[17];      // list count entering each level (lists[levels] == 1)
  int64_t klen[17];       // list length entering each level
  size_t ws_bytes;        // ping-pong scratch for intermediate levels
};
int plan_merge(int64_t nq, int64_t nlists, int64_t kin, int64_t k, MergePlan* p);
// out_dist/out_row may be null; out_kth (optional) receives each query's k-th
// smallest composite (kEmpty if fewer than k candidates).
// gate/gate_cap: as ScanArgs::gate, per query of the merge.
// count (optional): appended lists, query q's entries are its first
// count[q * kCountStride] slots (capped at nlists * kin; the rest unread).
// zero_count: reset each query's count once read (only a one-level plan,
// where one workgroup per query reads it; ignored otherwise).
int run_merge(const MergePlan& p, const uint64_t* in, int64_t nq, int64_t k, void* ws,
              float* out_dist, int64_t* out_row, hipStream_t stream,
              uint64_t* out_kth = nullptr, const uint32_t* gate = nullptr,
              int64_t gate_cap = 0, uint32_t* count = nullptr, bool zero_count = false);

// Batched queries (knn_batch.hip): fp32 MFMA GEMM + threshold filter.
struct BatchArgs {
  const float* X;         // [n][d] f32 corpus shard
  int64_t n;
  int d;
  int64_t row_base;
  const float* Q;         // [nq][d]
  const float* qnorm;     // [nq] max(|q|, 1e-12) (cosine) / sum q^2 (L2)
  int64_t nq;
  const uint32_t* mask;
  int64_t tile_start, tile_stride, num_tiles;  // which 128-row tiles to scan
  const uint64_t* thr;    // [nq] append rows whose composite <= thr
  uint32_t* count;        // [nq * kCountStride] appends (may exceed cap: overflow)
  uint64_t* cand;         // [nq][cap]
  int cap;
  float l2_eps;           // L2: relative error bound of |x|^2+|q|^2-2x.q in fp32
};
int launch_batch(const BatchArgs& a, int metric, hipStream_t stream);
// mode 0: max(|q|, 1e-12) (cosine); mode 1: sum q^2 (L2 expansion)
int launch_qnorm(const float* Q, int64_t nq, int d, float* out, hipStream_t stream,
                 int mode = 0);
// Replace each candidate's key by its exact distance (the single-query scan's
// summation order: bit-identical).  thr (optional): candidates whose key is
// above the query's thr key are dropped (kEmpty) without being read.
// qnorm: cosine only, max(|q|, 1e-12) as the scan computes it.
int launch_rescore(const void* X, int dtype, int64_t n, int d, int64_t row_base,
                   const float* Q, const float* qnorm, int64_t nq, const uint32_t* count,
                   uint64_t* cand, int cap, int metric, const uint64_t* thr, hipStream_t stream);
// thr[q] = min(thr[q], the largest exact composite of the query's k rows
// [nq][k] (global, -1 = missing: the query keeps its threshold)); scratch
// [nq][2] uint64 zeroed before the first call (left zeroed by each call)
int launch_exact_kth(const void* X, int dtype, int64_t n, int d, int64_t row_base,
                     const float* Q, const float* qnorm, int64_t nq, int k, int64_t* rows,
                     int metric, uint64_t* thr, hipStream_t stream);

// run_merge (top-k by key of each query's first count[q] entries of keys
// [nq][cap]) + launch_exact_kth in one launch, any cap (knn_batch.hip
// select_kernel, streaming over LDS-sized chunks)
// prune (these three): scratch of select_prune_bytes(nq, k, cap) or null;
// a plan that prunes (k ~ 1 000 over a large buffer) first keeps the k
// smallest of every LDS-sized slice in parallel (select_kernel MODE 3)
int select_prune_lists(int64_t k, int64_t cap);
size_t select_prune_bytes(int64_t nq, int64_t k, int64_t cap);
int launch_exact_threshold(const void* X, int dtype, int64_t n, int d, int64_t row_base,
                           const float* Q, const float* qnorm, int64_t nq, const uint64_t* keys,
                           int64_t cap, uint32_t* count, bool zero_count, int k, int metric,
                           uint64_t* thr, hipStream_t stream, uint64_t* prune = nullptr,
                           int64_t* topr = nullptr, const uint64_t* gate_cand = nullptr,
                           int64_t gate_num = 0, int64_t gate_den = 1);
// (gate_cand: launch_overflow_gate(gate_cand, count, thr, nq, cap, gate_num,
// gate_den) follows on the new thresholds, fused into the select's workgroups
// when the select computes them itself)
// thr[q] = min(thr[q], the k-th smallest of the query's first count[q] keys)
// when it has at least k (run_merge's threshold-only level, any cap)
int launch_sample_threshold(const uint64_t* keys, int64_t nq, int64_t cap, uint32_t* count,
                            bool zero_count, int k, uint64_t* thr, hipStream_t stream,
                            uint64_t* prune = nullptr);
// the final top-k of each query's first count[q] exact composites of keys
// [nq][cap], sorted and decoded (run_merge's last level, one workgroup per
// query, any cap); a query whose count exceeds alt_gate selects from its
// alt_m entries of alt ([nq][alt_m], the overflow fallback scan's lists)
int launch_final_select(const uint64_t* keys, int64_t nq, int64_t cap, const uint32_t* count,
                        int k, float* out_dist, int64_t* out_row, const uint64_t* alt,
                        int64_t alt_m, int64_t alt_gate, hipStream_t stream,
                        uint64_t* prune = nullptr);

// Batched filter on the fp16 matrix cores (knn_filter.hip): appends every
// (row, query) whose rigorous lower bound reaches the query's threshold.
struct FilterArgs {
  const void* X;          // [n][d] corpus shard (f32 or f16)
  int dtype;              // FX_DTYPE_F32 / FX_DTYPE_F16
  int64_t n;
  int d;
  int64_t row_base;
  const uint16_t* Qh;     // fp16 queries scaled by a power of two, in blocks of 32
                          // components: (q, k) at ((k / 32) * qstride + q) * 32 + k % 32
  int dq;                 // components per query, padded (a multiple of 64)
  int64_t qstride;        // queries per block row (nq_pad)
  const float* qinfo;     // [nq][4] {1/scale, norm term, A, B}
  int64_t nq;
  const uint32_t* mask;
  int64_t tile_start, tile_stride, num_tiles;  // which 256-row tiles to scan
  const uint64_t* thr;    // [nq] append when order_key(lb) <= thr >> 32
  uint32_t* count;        // [nq * kCountStride] appends (may exceed cap: overflow)
  uint64_t* cand;         // [nq][cap] ub composites (cand_ub null) or lb composites
  uint64_t* cand_ub;      // [nq][cap] ub composites, or null (sampling phases)
  int cap;
  const float* rowinfo;   // [n] row sums of squares of the f32 rows when X is their fp16
                          // filter image (dtype F16), NaN = forced; null otherwise;
                          // img8: [n][kI8RowInfo] (launch_image8)
  int img8;               // X is the int8 filter image (launch_image8), Qh/qinfo from
                          // launch_qprep8
  int all_pass;           // no query has a threshold yet (thr all empty): img8 appends
                          // every live pair without the test
  int skip_full;          // a workgroup whose queries all hold count > cap returns at once
  uint64_t perm_a;        // img8: image row i holds corpus row (perm_a * i) % n (image8_perm)
  int ub_test;            // sampling phase after the first: append when the UPPER bound
                          // reaches the threshold (only the k-th upper bound is needed)
  int diag;               // FX_FILTER_DIAG (diagnostic builds only): 1 no appends, 2 no epilogue,
                          // 4 no MFMA, 8 no query loads, 16 no LDS stores,
                          // 32 no append atomics, 64 no append stores
};
int launch_filter(const FilterArgs& a, int metric, hipStream_t stream);
// the LDS-DMA ring variant (knn_filter.hip ring_kernel) with FX_FILTER_RING=1
// (the register-staged kernel otherwise)
bool filter_ring();
// filter images in MFMA fragment order (knn_filter.hip filter_img2_kernel);
// FX_IMAGE_TILED=0: row-major
bool image_tiled();
// int8 filter images (knn_filter.hip): per row kI8RowInfo floats {w, 1/s,
// N/s, n2/s, 0...} (launch_image8), per query kI8QInfo floats {s_q, R', n_q^2,
// |q|, 0...} (launch_qprep8); kI8Kappa bounds P/R' (the two query error terms,
// see knn_filter.hip "int8 filter image")
constexpr int kI8RowInfo = 4;
constexpr int kI8QInfo = 4;
constexpr float kI8Kappa = 128.f;
int launch_image8(const void* X, int dtype, int64_t n, int d, void* img, float* rowinfo,
                  hipStream_t stream);
// The int8 image stores its rows in the order of an affine permutation of the
// corpus: image row i holds corpus row (a * i) % n, a ~ 0.618 n coprime with n
// (a Weyl sequence).  The filter's nested samples take every r-th tile of the
// IMAGE, so they are equidistributed over the corpus whatever its order: a
// corpus stored in clusters (the reference test's x + 10 x0 per 1 000-row
// batch) or sorted by any key no longer hides its nearest rows from the
// samples.  1 for n <= 2.
uint64_t image8_perm(int64_t n);
__device__ __forceinline__ uint32_t perm_row(uint64_t a, int64_t n, int64_t i) {
  return (uint32_t)((a * (uint64_t)i) % (uint64_t)n);
}
// Final-pass overflow prediction (img8): per query, the appended candidates of
// the last sample (count, cand: lb composites) that pass the new threshold thr,
// scaled by num / den (the remaining tiles over the sample's), plus count: a
// query predicted to exceed cap gets count = cap + 1 (the final pass skips it
// and the exact scan recomputes it, fx_knn_reduce's gated fallback)
int launch_overflow_gate(const uint64_t* cand, uint32_t* count, const uint64_t* thr, int64_t nq,
                         int cap, int64_t num, int64_t den, hipStream_t stream);
// (thr, count: when given, each query's threshold is set empty and its append
// count zeroed in the same launch)
int launch_qprep8(const float* Q, int64_t nq, int64_t nq_pad, int d, int dq, int metric,
                  int8_t* Qb, float* qinfo, hipStream_t stream, uint64_t* thr = nullptr,
                  uint32_t* count = nullptr);
int launch_qprep(const float* Q, int64_t nq, int64_t nq_pad, int d, int dq, int metric,
                 uint16_t* Qh, float* qinfo, hipStream_t stream);
int filter_tile_rows(int dtype);
// fp16 filter image + row sums of squares of an f32 corpus (knn_filter.hip)
int launch_image(const float* X, int64_t n, int d, void* img, float* rowinfo, hipStream_t stream);
int filter_query_pad(int64_t nq);
int filter_dq(int d);
int batch_tile_rows();
int launch_encode(const float* dist, const int64_t* row, int64_t count, uint64_t* out,
                  hipStream_t stream);
int launch_fill(void* x, int dtype, int64_t n, int64_t d, uint64_t seed, int64_t row_base,
                int64_t cluster, hipStream_t stream);

// error / device helpers (capi.hip)
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
int check_launch(const char* what);
int device_cus(int* out);
int kernel_occupancy(const void* fn, int block, size_t smem, int* out);
// raise the dynamic-LDS limit of fn to 160 KB on the current device (once per device)
int allow_lds(const void* fn);

// k above the fused path (knn_large.hip): all distances + radix sort.
struct LargeLayout {
  size_t off_dist, off_keys, off_sorted, off_temp, temp_bytes, total;
};
LargeLayout plan_large(int64_t n, int64_t nq);
// distances (distance-mode scan with plan p) + composites into ws
int large_scan(const ScanPlan& p, ScanArgs a, int64_t nq, const LargeLayout& l, char* ws,
               hipStream_t st);
int large_reduce(int64_t n, int64_t nq, int64_t k, const LargeLayout& l, char* ws,
                 float* out_dist, int64_t* out_row, hipStream_t st);

}  // namespace fx
