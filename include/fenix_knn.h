/*
 * fenix_knn.h — C ABI of the MI355X (gfx950) brute-force kNN engine behind
 * fenix's search path.
 *
 * Reference path replaced (nrlugg/fenix, paths relative to /root/reference):
 *   src/fenix/flight.py:242-288        Flight.search (client, unchanged API)
 *   src/fenix/flight.py:62-77          Server.do_exchange → io.index.call
 *   src/fenix/io/index/index.py:81-170 io.index.call (brute-force branch, coding=None)
 *   src/fenix/io/index/index.py:133-162  per-chunk scalar UDF "distance:{metric}:{T}:{D}"
 *   src/fenix/io/coder/coder.py:38-50  io.coder.distance (cdist / -u@v / cosine)
 *   src/fenix/io/index/index.py:165-168  pc.select_k_unstable + Table.take
 *
 * The reference's pluggable boundary is Python-level (io.index.call and the
 * pyarrow compute-function registry).  The host mirror in fenix_amd/ binds
 * these entry points with ctypes.  All pointers are
 * device pointers unless stated otherwise; all calls are asynchronous on the
 * given hipStream_t (passed as void*), borrow their inputs, allocate nothing
 * per call, and operate on the calling thread's current HIP device.
 *
 * Ordering contract (deterministic tie-break): results are the k smallest
 * (distance, global_row) pairs, ascending by distance then by row.  -0.0 is
 * treated as +0.0; NaN distances order after every number (Arrow
 * select_k_unstable: NaN after numbers).  A slot with no candidate (fewer than
 * k admissible rows) returns distance NaN and row -1.
 *
 * Row numbering: global_row = row_base + local_row; global rows must be
 * < 2^32 - 1 (4.29 G rows per search).
 *
 * Return value of every int function: 0 on success, negative on failure; the
 * message is available from fx_last_error() (thread-local).
 */
#ifndef FENIX_KNN_H
#define FENIX_KNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* dtype of the corpus (the Arrow fixed_size_list value type) */
#define FX_DTYPE_F32 0
#define FX_DTYPE_F16 1
#define FX_DTYPE_QU8 2     /* uint8 codes, value = scale * (code - zero_point):
                              the quint8 tensor column of ex/arrow/quint8/quint8.py:56-145;
                              fx_knn_*_ex entry points only */

/* metric; aliases are resolved by the host (coder.py:39 "euclidean"->l2,
 * coder.py:47 "dot"->inner_product) */
#define FX_METRIC_L2 0     /* sqrt(sum (x-q)^2)                      coder.py:39-40 */
#define FX_METRIC_IP 1     /* -(x . q)                               coder.py:47-48 */
#define FX_METRIC_COS 2    /* 0.5 - 0.5 (x/max|x|,1e-12).(q/max|q|)  coder.py:42-45 */

/* error codes */
#define FX_OK 0
#define FX_EINVAL -1       /* bad argument (maps to ValueError / AssertionError) */
#define FX_EUNSUPPORTED -2 /* valid but not supported by this build */
#define FX_EHIP -3         /* HIP runtime failure (maps to RuntimeError) */

/* ABI version (major*100 + minor). */
int fx_version(void);

/* Thread-local description of the last failure on this thread. */
const char* fx_last_error(void);

/* Number of visible HIP devices. */
int fx_device_count(int* out);

/*
 * Process-wide options, set explicitly by the host.  The library reads no
 * environment variable: a serving process's kernel selection cannot change
 * through its environment.  Name, default, meaning:
 *   "batched"             1  0: each query of a batch runs the single-query scan
 *   "batch_min_queries"   2  smallest batch that takes the batched filter (1:
 *                            single float32 queries too, with a filter image)
 *   "filter_image"        8  which filter image a host builds for float32
 *                            corpora: 8 (fx_filter_image8), 16
 *                            (fx_filter_image) or 0 (none); read by the host
 *                            (fenix_amd.engine), not by the library's calls
 * Test switches (they change which code runs, never the results):
 *   "batch_cap"           0  candidate buffer per query of the batched filter
 *                            (0: max(64 k, 16 K); smaller than 16 k is ignored)
 *   "batch_sample_ratio"  0  row-sample ratio of the filter phases (0: cap / 4k,
 *                            8 with an int8 image; up to cap / 4k accepted)
 *   "batch_ub_test"       1  sampling phases append the pairs whose upper
 *                            bound reaches the threshold (0: lower bound)
 *   "single_query_image"  1  0: single queries keep the exact scan even when
 *                            an int8 filter image is supplied
 *   "i8_max_k"         1024  largest k an int8 filter image serves (larger k:
 *                            the fp16 image / f32 rows, or the exact scan);
 *                            at most 2048 (FX_EINVAL above)
 *   "img6"                1  1: int8-image batches of <= 128 queries (single
 *                            queries included) run the resident-query-slice
 *                            kernel; 2: larger batches too (as several
 *                            slices); 0: every batch the streamed-query-tile
 *                            kernel
 *   "img8"                1  1: int8-image batches of > 128 queries with d <= 768
 *                            run the queries-in-registers kernel (except the
 *                            all-pass first sample); 0: the streamed-query-tile
 *                            kernel
 *   "i8_sample_ratio"     8  int8 images: the final pass's sample F1 holds every
 *                            r1-th tile (at least 2, at most cap / 4k)
 *   "i8_grow_ratio"      16  int8 images: each sample before F1 is r2 times
 *                            smaller than the next (at least 2, at most cap / 4k)
 *   "select_prune"        1  int8 images: the selects over the candidate buffer
 *                            first keep the k smallest of each 16 K slice in
 *                            parallel when k >= 512 (2: at any k; 0: never)
 *   "force_fallback"      0  1: every batched query is recomputed by the exact
 *                            single-query scan, as if its candidates overflowed
 *   "scan_interleave"    -1  -1: by row size; 0: one row range per workgroup;
 *                            1: block steps dealt round-robin over the grid
 *   "q8_dma"              1  0: quint8 scans without the LDS-DMA ring
 * fx_set_option: FX_EINVAL for an unknown name.  Options are read when a call
 * plans its launches; set them while no search is in flight.
 */
int fx_set_option(const char* name, int64_t value);
int fx_get_option(const char* name, int64_t* out);

/*
 * Host-blocking synchronisations (stream / device synchronise, blocking copy)
 * the library has performed since it was loaded.  Every entry point is
 * asynchronous on its stream, so searches leave this count unchanged; tests
 * assert that, e.g. across a search over shards on several devices.
 */
uint64_t fx_host_sync_count(void);

/* Largest k of the fused scan + merge path (1024).  Any larger k (the
 * reference's maxval is unbounded, index.py:165-168) is served by a
 * distance-mode scan + radix sort of all n composites (knn_large.hip): every
 * search entry point and fx_topk_merge accept k up to 2^31 - 1, with the same
 * ordering contract, at the cost of n*nq*20 bytes of workspace. */
int64_t fx_max_k(void);

/*
 * Workspace needed by fx_knn_search for this shape on the current device.
 * Replaces nothing in the reference directly: the reference allocates an
 * n-row distance column per call (index.py:162); this engine needs only
 * candidate lists, O(nq * lists * k) bytes.
 */
int fx_knn_workspace_bytes(int64_t n, int64_t d, int dtype, int64_t nq, int64_t k,
                           size_t* out_bytes);
/*
 * The same for a search that is (img8 = 1) or is not (img8 = 0) given an int8
 * filter image (fx_knn_scan_img8 / fx_knn_search_img8 with a non-null image).
 * An int8-image plan holds 4x the candidate buffers of the image-free one;
 * fx_knn_workspace_bytes is the img8 = 1 answer, enough for either.
 */
int fx_knn_workspace_bytes_img8(int64_t n, int64_t d, int dtype, int64_t nq, int64_t k,
                                int img8, size_t* out_bytes);

/*
 * Exact k-nearest-neighbour search of nq queries over one row-major corpus
 * shard [n][d] of dtype.  Replaces index.py:162-168 (distance UDF over every
 * chunk + select_k_unstable) for coding=None.
 *   corpus   device, n*d elements of dtype, row-major (the Arrow values buffer)
 *   row_base global row number of corpus row 0 (multi-source / multi-GPU shards)
 *   queries  device, nq*d float32 (already cast to the column type: index.py:111)
 *   mask     device bitmap over local rows (bit r of word r>>5), 1 = row is
 *            admissible; NULL = all rows (replaces data.filter, index.py:161)
 *   out_dist device [nq][k] float32, out_row device [nq][k] int64
 */
int fx_knn_search(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                  const float* queries, int64_t nq, int metric, int64_t k,
                  const uint32_t* mask, void* ws, size_t ws_bytes, float* out_dist,
                  int64_t* out_row, void* stream);

/*
 * fx_knn_search in two phases, for callers that overlap or time them apart:
 * fx_knn_scan launches the scan kernels (candidates into ws); fx_knn_reduce
 * launches the merge that turns them into out_dist / out_row.  Both must be
 * given the same arguments.
 * Batched queries (nq >= 2, float32 rows with d % 4 == 0 or float16 rows
 * with d % 8 == 0, 16-B aligned corpus, any metric) take the matrix-core
 * path: fx_knn_scan runs the sampled-threshold phases of the fp16-MFMA bound
 * filter and rescores the surviving candidates exactly, so the results are
 * bit-identical to the single-query scan; fx_knn_reduce recomputes any
 * query whose candidates overflowed with the exact single-query scan, decided
 * on the device: the fallback launches read the per-query candidate counts
 * and their workgroups return at once for queries that did not overflow, so
 * no call synchronises with the host and the whole search can be queued on
 * several devices back to back (or captured in a graph).
 */
int fx_knn_scan(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                const float* queries, int64_t nq, int metric, int64_t k,
                const uint32_t* mask, void* ws, size_t ws_bytes, void* stream);
int fx_knn_reduce(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                  const float* queries, int64_t nq, int metric, int64_t k,
                  const uint32_t* mask, void* ws, size_t ws_bytes, float* out_dist,
                  int64_t* out_row, void* stream);

/*
 * fp16 filter image of a float32 corpus, a resident companion of the corpus
 * (HBM is 288 GB per GPU; the image is half the corpus).  fx_filter_image
 * writes image [n][d] fp16 (each component rounded to nearest, as the batched
 * filter converts it) and rowinfo [n] float32 (the row's sum of squares; NaN
 * marks a row the filter must pass: non-finite, or a component that overflows
 * fp16).  d must be a multiple of 8; corpus and image 16-B aligned.  The
 * image must be rebuilt whenever the corpus changes.
 * fx_knn_scan_img / fx_knn_search_img = fx_knn_scan / fx_knn_search (same
 * workspace, same results bit for bit; fx_knn_reduce completes either) whose
 * batched filter phases stream the image instead of the float32 rows; the
 * candidates are still rescored from the float32 rows.  fx_filter_image_used
 * says whether a search of that shape reads the image at all (batched
 * float32 queries through the filter), so a caller builds it only then.
 * Replaces nothing in the reference: the per-chunk UDF reads the float32
 * column every time (src/fenix/io/index/index.py:137-162).
 */
int fx_filter_image_bytes(int64_t n, int64_t d, size_t* image_bytes, size_t* rowinfo_bytes);
int fx_filter_image(const float* corpus, int64_t n, int64_t d, void* image, float* rowinfo,
                    void* stream);
int fx_filter_image_used(int64_t n, int64_t d, int dtype, int64_t nq, int64_t k, int metric,
                         int* out);
int fx_knn_scan_img(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                    const void* image, const float* rowinfo, const float* queries, int64_t nq,
                    int metric, int64_t k, const uint32_t* mask, void* ws, size_t ws_bytes,
                    void* stream);
int fx_knn_search_img(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                      const void* image, const float* rowinfo, const float* queries, int64_t nq,
                      int metric, int64_t k, const uint32_t* mask, void* ws, size_t ws_bytes,
                      float* out_dist, int64_t* out_row, void* stream);

/*
 * int8 filter image of a float32 corpus: the same role as the fp16 image at a
 * quarter of the corpus bytes, searched on the int8 matrix cores (twice the
 * fp16 rate).  fx_filter_image8 writes image (row tiles of 32 rows in MFMA
 * fragment order, each row scaled to int8 by its own scale) and rowinfo [n][4]
 * float32 (the row's bound terms; NaN first term = forced through).  The
 * rigorous bounds are wider than fp16's, so the filter keeps more candidates
 * and refines its thresholds by exact rescoring; results are the same bits as
 * fx_knn_scan / fx_knn_search.  d must be a multiple of 8; corpus, image and
 * rowinfo 16-B aligned; same workspace as fx_knn_scan.  Rebuild whenever the
 * corpus changes.  Replaces nothing in the reference (see above).
 * With an image, a SINGLE query over a float32 corpus of >= 4 GiB also takes
 * the filter (option "single_query_image", default 1: 10M x 768 1.41 ms vs
 * the 4.34 ms scan); the scan's candidates then live in the filter's
 * workspace layout, so the two-call form pairs fx_knn_scan_img8 with
 * fx_knn_reduce_img8 (same image pointer), never with fx_knn_reduce.
 * fx_filter_image_used reports the single-query case when the "filter_image"
 * option is 8.
 */
int fx_filter_image8_bytes(int64_t n, int64_t d, size_t* image_bytes, size_t* rowinfo_bytes);
/* Row order of the int8 image: image row i (and rowinfo row i) holds corpus
 * row (mult * i) % n, an affine permutation (mult ~ 0.618 n, coprime with n),
 * so the filter's tile-strided samples are spread over the whole corpus even
 * when it is stored in clusters or sorted.  For tests and tools. */
int fx_filter_image8_perm(int64_t n, uint64_t* mult);
/* After a batched / filter-image search (fx_knn_scan*, before the workspace
 * is reused): each query's final candidate count (device uint32 [nq]) and
 * the buffer's capacity (*out_cap; -1 when the search did not run the
 * filter).  count > cap means the exact scan recomputed that query.  Same
 * shape arguments as the scan; img8 = 1 when it received an int8 image.
 * For tests and tools. */
int fx_knn_filter_counts(const void* corpus, int dtype, int64_t n, int64_t d, int64_t nq,
                         int metric, int64_t k, int img8, const void* ws, size_t ws_bytes,
                         uint32_t* out_counts, int64_t* out_cap, void* stream);
/* The same search's thresholds (device uint64 [nq] composites) and candidate
 * buffers (device uint64 [nq][cap]: lower-bound / exact composites, upper-
 * bound composites; each nullable).  For tests and tools. */
int fx_knn_filter_state(const void* corpus, int dtype, int64_t n, int64_t d, int64_t nq,
                        int metric, int64_t k, int img8, const void* ws, size_t ws_bytes,
                        uint64_t* out_thr, uint64_t* out_cand, uint64_t* out_cand_ub,
                        void* stream);
int fx_filter_image8(const float* corpus, int64_t n, int64_t d, void* image, float* rowinfo,
                     void* stream);
/* The same image of a float32 or float16 corpus (dtype FX_DTYPE_F32 /
 * FX_DTYPE_F16): an fp16 column's searches then stream 1 byte per component
 * instead of 2 and rescore from the fp16 rows in the fp16 scan's order. */
int fx_filter_image8_typed(const void* corpus, int dtype, int64_t n, int64_t d, void* image,
                           float* rowinfo, void* stream);
int fx_knn_scan_img8(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                     const void* image, const float* rowinfo, const float* queries, int64_t nq,
                     int metric, int64_t k, const uint32_t* mask, void* ws, size_t ws_bytes,
                     void* stream);
int fx_knn_search_img8(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                       const void* image, const float* rowinfo, const float* queries, int64_t nq,
                       int metric, int64_t k, const uint32_t* mask, void* ws, size_t ws_bytes,
                       float* out_dist, int64_t* out_row, void* stream);
int fx_knn_reduce_img8(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                       const void* image, const float* queries, int64_t nq, int metric, int64_t k,
                       const uint32_t* mask, void* ws, size_t ws_bytes, float* out_dist,
                       int64_t* out_row, void* stream);

/*
 * fx_knn_search over a list of corpus rows instead of all of them: rows
 * [nrows] int32 local row numbers (< n, device), e.g. the rows kept by a
 * filter or a probe set (fx_mask_compact).  The scan reads only the listed
 * rows, so a selective filter (index.py:161) or probe set (index.py:113-126)
 * costs its own bytes, not the corpus's.  Results use global rows
 * (row_base + listed row) and the same ordering contract; nrows >= 1.
 */
int fx_knn_search_rows_workspace_bytes(int64_t nrows, int64_t d, int dtype, int64_t nq,
                                       int64_t k, size_t* out_bytes);
int fx_knn_search_rows(const void* corpus, int dtype, int64_t n, int64_t d, int64_t row_base,
                       const int32_t* rows, int64_t nrows, const float* queries, int64_t nq,
                       int metric, int64_t k, void* ws, size_t ws_bytes, float* out_dist,
                       int64_t* out_row, void* stream);

/*
 * All distances of nq queries to every corpus row: out[nq][n] float32.
 * Replaces the per-chunk UDF / coder.distance (index.py:137-151, coder.py:38-50)
 * where the reference returns the whole table (maxval None or n <= maxval,
 * index.py:165).  Masked-out rows get NaN.
 */
int fx_knn_distances(const void* corpus, int dtype, int64_t n, int64_t d,
                     const float* queries, int64_t nq, int metric, const uint32_t* mask,
                     float* out, void* stream);

/*
 * Merge `parts` sorted top-k lists per query (e.g. one per GPU shard or per
 * source) into one: in_dist/in_row [nq][parts][kin] (device), out [nq][k].
 * Same ordering contract.  Replaces select_k over the concatenated table of
 * several sources (table.py:19-21 + index.py:166) and is the final merge
 * after the cross-GPU all-gather.
 */
int fx_topk_merge_workspace_bytes(int64_t nq, int64_t parts, int64_t kin, int64_t k,
                                  size_t* out_bytes);
int fx_topk_merge(const float* in_dist, const int64_t* in_row, int64_t nq, int64_t parts,
                  int64_t kin, int64_t k, void* ws, size_t ws_bytes, float* out_dist,
                  int64_t* out_row, void* stream);

/*
 * Portable synthetic corpus generator (test/bench data; bit-identical to
 * oracle/knn_ref.c fx_ref_fill): element (r, c) = IrwinHall4(splitmix64(
 * seed * 0x9E3779B97F4A7C15 + (row_base + r) * d + c)), approximately N(0,1).
 * The clustered variant (tests/test_flight.py:21-22 of the reference)
 * adds 10 * row[batch_start] to every row of each `cluster`-row batch
 * (cluster <= 0: plain).
 */
int fx_fill_normal(void* x, int dtype, int64_t n, int64_t d, uint64_t seed, int64_t row_base,
                   int64_t cluster, void* stream);

/*
 * Per-row sum of squares in f32: out[r] = sum_c x[r][c]^2 (x: [n][d] f32/f16).
 * The ||x||^2 term of the L2 expansion and the cosine norms (F.normalize,
 * coder.py:43-44, 55-56).
 */
int fx_row_sqnorms(const void* x, int dtype, int64_t n, int64_t d, float* out, void* stream);

/* ---------------------------------------------------------------- coded index
 * A coding (src/fenix/io/coder/coder.py:24-35) is nb = num_codebooks
 * independent codebooks of ks = codebook_size full-width f32 codewords,
 * codewords[nb][ks][d].  The composite code of a row is
 *     sum_j argmin_c dist(x, codewords[j][c]) * ks^(nb-1-j)
 * (coder.py:171-186 with maxval = 1, as index.make encodes a table,
 * index.py:37-65).  Ties go to the lowest codeword index.
 */

/*
 * Nearest codeword of every row in every codebook.  x: [n][d] corpus rows
 * (f32/f16).  Outputs (each nullable): out_index [n][nb] int32 codeword index,
 * out_code [n] int64 composite code (needs ks^nb < 2^31), out_dist [n][nb] f32
 * the metric's distance to the chosen codeword.  Replaces the per-batch
 * pc.call_function(coding, [x, 1]) of index.py:46-49 -> coder.call
 * (coder.py:143-194) and the argmin of coder.update (coder.py:58-59).
 */
int fx_code_assign_workspace_bytes(int64_t n, int64_t d, int64_t nb, int64_t ks,
                                   size_t* out_bytes);
int fx_code_assign(const void* x, int dtype, int64_t n, int64_t d, const float* codewords,
                   int64_t nb, int64_t ks, int metric, void* ws, size_t ws_bytes,
                   int32_t* out_index, int64_t* out_code, float* out_dist, void* stream);

/*
 * One mini-batch k-means step of every codebook, in place: the body of the
 * training loop, coding = vmap(update)(coding, sample) (coder.py:53-65, 118).
 * sample: [nb][bs][d] rows (f32/f16), slice j trains codebook j;
 * codewords: [nb][ks][d] f32, updated in place.  cosine: codewords and sample
 * rows are normalised first and the result is normalised again; every
 * codeword becomes the mean of itself and the rows assigned to it
 * (torch.index_reduce "mean", include_self), summed in row order.
 */
int fx_kmeans_step_workspace_bytes(int64_t nb, int64_t bs, int64_t d, int64_t ks,
                                   size_t* out_bytes);
int fx_kmeans_step(const void* sample, int dtype, int64_t nb, int64_t bs, int64_t d,
                   float* codewords, int64_t ks, int metric, void* ws, size_t ws_bytes,
                   void* stream);

/*
 * Probe selection (coder.py:171-186, index.py:113-121): cw_dist [nq][nb][ks]
 * holds each target's distance to every codeword (fx_knn_distances with the
 * codewords as the corpus); the composite score of code c is the sum over
 * j = 0..nb-1 (in that order, f32) of the distance to its digit j.  Emits the
 * `probes` best composites per target in (score, code) order: out_code
 * [nq][probes] int64, out_score [nq][probes] f32, out_sel [nq][ceil(ks^nb/32)]
 * bitmap of the selected codes (each nullable).  ks^nb * nq < 2^31.
 */
int fx_code_probe_workspace_bytes(int64_t nq, int64_t nb, int64_t ks, size_t* out_bytes);
int fx_code_probe(const float* cw_dist, int64_t nq, int64_t nb, int64_t ks, int64_t probes,
                  void* ws, size_t ws_bytes, int64_t* out_code, float* out_score,
                  uint32_t* out_sel, void* stream);

/*
 * Row bitmap of a probe search: bit r = (row_code[r] is set in sel) AND
 * (filter == NULL or bit r of filter).  The filter expression
 * pc.field("__CODED_ID__").isin(probe codes) & filter of index.py:117-126,
 * consumed as the `mask` of fx_knn_search.  out_mask: ceil(n/32) words;
 * out_count (nullable, one uint64 on the device): the number of rows kept —
 * len(data) after the filter, which decides maxval's branch (index.py:165).
 */
int fx_code_mask(const int64_t* row_code, int64_t n, const uint32_t* sel, int64_t ncodes,
                 const uint32_t* filter, uint32_t* out_mask, uint64_t* out_count, void* stream);

/*
 * Row bitmap -> ascending list of the set rows (int32), and their count
 * (out_count: one uint64 on the device, nullable).  Three passes, no atomics,
 * deterministic.  n < 2^31.
 */
int fx_mask_compact_workspace_bytes(int64_t n, size_t* out_bytes);
int fx_mask_compact(const uint32_t* mask, int64_t n, void* ws, size_t ws_bytes, int32_t* out_rows,
                    uint64_t* out_count, void* stream);

/* ------------------------------------------------------ corpus descriptor
 * The _ex entry points take the corpus as a descriptor, which also carries
 * the dequantisation of FX_DTYPE_QU8 columns (per-tensor affine quint8,
 * ex/arrow/quint8/quint8.py:56-58, 81-84: value = scale * (code - zero_point),
 * computed in f32 exactly as QUInt8NDArray.dequantize does), and an optional
 * row list (rows/nrows as in fx_knn_search_rows; rows == NULL: all n rows).
 * The queries stay float32 (asymmetric distances: only the corpus is coded).
 */
typedef struct fx_corpus {
  const void* data;    /* device, [n][d] of dtype */
  int dtype;           /* FX_DTYPE_F32 / F16 / QU8 */
  int64_t n, d;
  int64_t row_base;    /* global row of row 0 */
  float scale;         /* QU8 only */
  int32_t zero_point;  /* QU8 only */
} fx_corpus;

/*
 * Exact top-k over several row shards that live on ONE device (the sources
 * of a multi-source table, table.py:19-21, or several shards of one column
 * on one GPU) with ONE merge tree: every shard's fused scan writes its
 * per-block top-k lists into one buffer and a single merge selects the k
 * smallest (distance, global row) over all of them.  The per-shard form
 * (fx_knn_search per shard + fx_topk_merge) runs a merge tree per shard and
 * one more over the shards.  Replaces index.py:162-168 over concatenated
 * sources.  Shards: same d, one dtype of FX_DTYPE_F32 / F16 / QU8 (each
 * QU8 shard with its own scale and zero point), n >= 1, each with its own
 * row_base; masks: NULL, or one bitmap (or NULL) per
 * shard.  k <= fx_max_k().  Exact scan only (a caller with a filter image
 * keeps the per-shard calls).  Results equal the per-shard form bit for bit.
 */
int fx_knn_search_shards_workspace_bytes(const fx_corpus* shards, int nshards, int64_t nq,
                                         int64_t k, size_t* out_bytes);
int fx_knn_search_shards(const fx_corpus* shards, int nshards, const float* queries, int64_t nq,
                         int metric, int64_t k, const uint32_t* const* masks, void* ws,
                         size_t ws_bytes, float* out_dist, int64_t* out_row, void* stream);

int fx_knn_search_ex_workspace_bytes(const fx_corpus* c, int64_t nrows, int64_t nq, int64_t k,
                                     size_t* out_bytes);
int fx_knn_search_ex(const fx_corpus* c, const int32_t* rows, int64_t nrows,
                     const float* queries, int64_t nq, int metric, int64_t k,
                     const uint32_t* mask, void* ws, size_t ws_bytes, float* out_dist,
                     int64_t* out_row, void* stream);
int fx_knn_distances_ex(const fx_corpus* c, const float* queries, int64_t nq, int metric,
                        const uint32_t* mask, float* out, void* stream);

/* ------------------------------------------------------ multi-GPU exchange
 * Single-process communicator over RCCL (xGMI): one rank per listed device
 * (a serving process driving every GPU of a node).  fx_allgather_topk gathers
 * every rank's [nq][k] top-k list into every rank's all_dist/all_row
 * [ndev][nq][k] buffers (one grouped call, each rank on its own stream);
 * fx_topk_merge then reduces them.  Replaces the select over the concatenated
 * sources of the reference (table.py:19-21 + index.py:166) when the shards
 * live on several GPUs.  RCCL is loaded on first use (dlopen librccl.so.1);
 * without it these return FX_EUNSUPPORTED.  Arrays of per-rank pointers are
 * host arrays of device pointers; streams is a host array of hipStream_t.
 */
int fx_comm_init_all(int ndev, const int* devs, void** out_comm);
int fx_comm_destroy(void* comm);
int fx_allgather_topk(void* comm, const float* const* dist, const int64_t* const* row,
                      int64_t nq, int64_t k, float* const* all_dist, int64_t* const* all_row,
                      void* const* streams);

#ifdef __cplusplus
}
#endif

#endif /* FENIX_KNN_H */
