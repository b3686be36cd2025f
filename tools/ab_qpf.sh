#!/bin/bash
# Query chunks two steps ahead in the tiled-image filter (FX_I2_QPF=2,
# libfenix_knn_qp2.so): parity with the variant, then same-box A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
FENIX_AMD_LIB=$PWD/fenix_amd/lib/libfenix_knn_qp2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -p no:cacheprovider -k "filter_image or batched or single_query_through" > gpurun_out/qpf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/qpf_tests.log
[ $rc -eq 0 ] || exit $rc
LIBS="new qp2" bash tools/ab_libs.sh --nq 256 --metric cosine || exit 1
LIBS="new qp2" bash tools/ab_libs.sh --nq 256 --metric l2 || exit 1
LIBS="new qp2" bash tools/ab_libs.sh --nq 16 --metric l2
