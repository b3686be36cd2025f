#!/bin/bash
# Row sums loaded at the tile start in the tiled-image filter (default on; rp0 = FX_I2_RPF=0,
# libfenix_knn_rp0.so): parity with the default build, then same-box A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -p no:cacheprovider -k "filter_image or batched or single_query_through" > gpurun_out/qpf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/qpf_tests.log
[ $rc -eq 0 ] || exit $rc
LIBS="new rp0" bash tools/ab_libs.sh --nq 256 --metric cosine || exit 1
LIBS="new rp0" bash tools/ab_libs.sh --nq 256 --metric l2 || exit 1
LIBS="new rp0" bash tools/ab_libs.sh --nq 16 --metric l2
