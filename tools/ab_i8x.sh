#!/bin/bash
# A/B: filter_img3_kernel image-stage depth (FX_I3_XS stages, FX_I3_XPF
# cross-tile prefetch) for the int8 and fp16 images, configs[2]; the product
# build first (correctness of the two-phase exact thresholds).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "filter_image or batched or overflow" > gpurun_out/i8x_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/i8x_tests.log; exit 1; }
tail -1 gpurun_out/i8x_tests.log
for rep in 1 2; do
  for v in new x3p1 x4p1 x4p0; do
    if [ "$v" = new ]; then unset FENIX_AMD_LIB; else export FENIX_AMD_LIB=$PWD/fenix_amd/lib/libfenix_knn_$v.so; fi
    for b in 8 16; do
      timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --nq 256 --metric cosine --opt filter_image=$b > gpurun_out/i8x_b.json 2>gpurun_out/i8x_b.err || { echo "bench failed $v"; tail -5 gpurun_out/i8x_b.err; exit 1; }
      python -c "import json;r=json.load(open('gpurun_out/i8x_b.json'));print('$v bits=$b', round(r['ms_per_step'],3), round(r['roofline']['kernel_ms'],3))"
    done
  done
done
unset FENIX_AMD_LIB
bash tools/prof_i8.sh > /dev/null
python tools/timeline.py gpurun_out/prof_i8_trace.csv qprep8 > gpurun_out/prof_i8_timeline.txt
cat gpurun_out/prof_i8_timeline.txt
