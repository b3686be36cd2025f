#!/bin/bash
# LDS append segments (FX_I2_SEG) on the GPU box: batched parity tests with the
# default library, then same-box A/B against variant builds (ABLIBS, e.g. s0 =
# fenix_amd/lib/libfenix_knn_s0.so built with UFLAGS=-DFX_I2_SEG=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -p no:cacheprovider -k "filter_image or batched or single_query_through" > gpurun_out/seg_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/seg_tests.log
[ $rc -eq 0 ] || exit $rc
LIBS="new ${ABLIBS:-s0}" bash tools/ab_libs.sh --nq 256 --metric cosine || exit 1
LIBS="new ${ABLIBS:-s0}" bash tools/ab_libs.sh --nq 16 --metric l2 || exit 1
LIBS="new ${ABLIBS:-s0}" bash tools/ab_libs.sh --nq 256 --metric l2
