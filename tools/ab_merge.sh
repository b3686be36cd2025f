#!/bin/bash
# A/B: one-level threshold merges (FX_MERGE_ENTRIES 16384, product) vs two
# levels of 8 K (libfenix_knn_m8.so), configs[2] cosine and L2, after the
# batched/image GPU tests on the product build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "filter_image or batched or overflow or merge" > gpurun_out/abm_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/abm_tests.log; exit 1; }
tail -1 gpurun_out/abm_tests.log
for rep in 1 2; do
  for v in new m8; do
    if [ "$v" = new ]; then unset FENIX_AMD_LIB; else export FENIX_AMD_LIB=$PWD/fenix_amd/lib/libfenix_knn_$v.so; fi
    for m in cosine l2; do
      timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --nq 256 --metric $m > gpurun_out/abm.json 2>gpurun_out/abm.err || { echo "bench failed $v"; tail -5 gpurun_out/abm.err; exit 1; }
      python -c "import json;r=json.load(open('gpurun_out/abm.json'));print('$v $m', round(r['ms_per_step'],3), round(r['roofline']['kernel_ms'],3))"
    done
  done
done
unset FENIX_AMD_LIB
