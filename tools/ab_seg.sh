#!/bin/bash
# LDS append segments (FX_I2_SEG) on the GPU box: batched parity tests with the
# variant library, then same-box A/B against the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
V=${V:-g32}
FENIX_AMD_LIB=$PWD/fenix_amd/lib/libfenix_knn_$V.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -p no:cacheprovider -k "filter_image or batched or single_query_through" > gpurun_out/seg_tests.log 2>&1
rc=$?; echo "tests ($V) rc=$rc"; tail -3 gpurun_out/seg_tests.log
[ $rc -eq 0 ] || exit $rc
LIBS="new ${ABLIBS:-g32 g16}" bash tools/ab_libs.sh --nq 256 --metric cosine || exit 1
LIBS="new ${ABLIBS:-g32 g16}" bash tools/ab_libs.sh --nq 16 --metric l2 || exit 1
LIBS="new ${ABLIBS:-g32 g16}" bash tools/ab_libs.sh --nq 256 --metric l2
