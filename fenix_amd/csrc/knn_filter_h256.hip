// The batched filter for fp16 rows and > 64 queries (knn_filter.hip compiled
// again, 64-wide K chunks): a row's K chunk is then 128 B, one whole cache
// line per row and load, where 32-wide chunks fetch every line twice.
#define FX_FILTER_VARIANT
#define FX_FILTER_BK 64
#define FX_FILTER_IMPL h256
#include "knn_filter.hip"
