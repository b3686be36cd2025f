#!/bin/bash
# A/B of the configs[2] batched filter: the product library (filter_img3_kernel,
# query ring by LDS-DMA) against a build with -DFX_FILTER_IMG3=0
# (filter_img2_kernel), same box, alternating.  Correctness first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 300 \
  -k "batched or filter_image or single_query_through or fp16" > gpurun_out/i3_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/i3_tests.log; exit 1; }
tail -3 gpurun_out/i3_tests.log
for rep in 1 2; do
  for v in new i2; do
    if [ "$v" = new ]; then unset FENIX_AMD_LIB; else export FENIX_AMD_LIB=$PWD/fenix_amd/lib/libfenix_knn_$v.so; fi
    for args in "--nq 256 --metric cosine" "--nq 256 --metric l2" "--nq 256 --metric inner_product"; do
      timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $args > gpurun_out/i3_b.json 2>gpurun_out/i3_b.err || { echo "bench failed $v $args"; tail -5 gpurun_out/i3_b.err; exit 1; }
      python -c "import json;r=json.load(open('gpurun_out/i3_b.json'));print('$v', '$args', round(r['ms_per_step'],3), round(r['roofline']['kernel_ms'],3), round(r['roofline']['frac'],3))"
    done
  done
done
unset FENIX_AMD_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -q -x --timeout 300 -k "batched" > gpurun_out/i3_full.log 2>&1; echo "fullsize rc $?"; tail -3 gpurun_out/i3_full.log
