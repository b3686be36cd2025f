#!/bin/bash
# 256-query image filter: 64-wide (default) vs 32-wide K chunks in the h256
# build (FX_H256_BK=32, libfenix_knn_bk32.so) and 32-wide with LDS append
# segments (libfenix_knn_bk32s.so): parity with the variant, then A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for V in bk32s; do
FENIX_AMD_LIB=$PWD/fenix_amd/lib/libfenix_knn_$V.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -p no:cacheprovider -k "filter_image or batched" > gpurun_out/bk_tests.log 2>&1
rc=$?; echo "tests ($V) rc=$rc"; tail -2 gpurun_out/bk_tests.log
[ $rc -eq 0 ] || exit $rc
done
LIBS="new bk32 bk32s" bash tools/ab_libs.sh --nq 256 --metric cosine || exit 1
LIBS="new bk32 bk32s" bash tools/ab_libs.sh --nq 256 --metric l2
