// The batched filter with 128-query tiles (knn_filter.hip compiled again):
// batches of 65..128 queries, which a 256-query tile would half pad.  K chunks
// of 32 (one 16-B query piece per thread), every row type and the tiled image.
#define FX_FILTER_VARIANT
#define FX_FILTER_BQ 128
#define FX_FILTER_BK 32
#define FX_FILTER_ROWS 3
#define FX_FILTER_IMPL q128
#include "knn_filter.hip"
