// filter_img3_kernel with 64-query tiles (knn_filter.hip compiled again, K
// chunks of 32 as the tiled images need): int8 filter images for batches of
// <= 64 queries, which a 256-query tile would multiply mostly as padding.
// Only its tiled-image kernel is compiled (fp16 and f32 rows of <= 64
// queries take the q64 build).
#define FX_FILTER_VARIANT
#define FX_FILTER_BQ 64
#define FX_FILTER_BK 32
#define FX_FILTER_ROWS 0  // the tiled-image kernel only
#define FX_FILTER_IMG3 1
#define FX_FILTER_IMPL q64i
#include "knn_filter.hip"
