#!/bin/bash
# A/B: filter_img3_kernel image-stage depth (FX_I3_XS stages, FX_I3_XPF
# cross-tile prefetch) against the product build, configs[2].
set -o pipefail
mkdir -p gpurun_out
for v in x3p0 x4p0; do
  FENIX_AMD_LIB=$PWD/fenix_amd/lib/libfenix_knn_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 300 \
    -k "batched_filter or filter_image or single_query_through or overflow" > gpurun_out/i3x_tests_$v.log 2>&1 || { echo "tests failed $v"; tail -30 gpurun_out/i3x_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/i3x_tests_$v.log)"
done
for rep in 1 2; do
  for v in new x3p0 x4p0; do
    if [ "$v" = new ]; then unset FENIX_AMD_LIB; else export FENIX_AMD_LIB=$PWD/fenix_amd/lib/libfenix_knn_$v.so; fi
    for m in cosine l2; do
      timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --nq 256 --metric $m > gpurun_out/i3x_b.json 2>gpurun_out/i3x_b.err || { echo "bench failed $v"; tail -5 gpurun_out/i3x_b.err; exit 1; }
      python -c "import json;r=json.load(open('gpurun_out/i3x_b.json'));print('$v $m', round(r['ms_per_step'],3), round(r['roofline']['kernel_ms'],3))"
    done
  done
done
