// The batched filter for fp16 rows (and f32 rows through their fp16 filter
// image) and > 64 queries (knn_filter.hip compiled again, 64-wide K chunks):
// a row's K chunk is then 128 B, one whole cache line per row and load, where
// 32-wide chunks fetch every line twice.  FX_H256_BK / FX_H256_WAVES are
// tuning knobs of this compilation only.
#define FX_FILTER_VARIANT
#ifndef FX_H256_BK
#define FX_H256_BK 64
#endif
#ifdef FX_H256_WAVES
#define FX_FILTER_WAVES FX_H256_WAVES
#endif
#define FX_FILTER_BK FX_H256_BK
#define FX_FILTER_ROWS 2
#define FX_FILTER_IMPL h256
#include "knn_filter.hip"
