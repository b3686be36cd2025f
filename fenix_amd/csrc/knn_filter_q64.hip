// The batched filter with 64-query tiles (knn_filter.hip compiled again):
// batches of <= 64 queries (e.g. concurrent requests coalesced by the Flight
// server, fenix_amd/coalesce.py) re-read and multiply a quarter of the padding.
#define FX_FILTER_VARIANT
#define FX_FILTER_BQ 64
#define FX_FILTER_IMPL q64
#include "knn_filter.hip"
