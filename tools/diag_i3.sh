#!/bin/bash
# Where the configs[2] filter's time goes (diagnostic build, FX_FILTER_DIAG
# switches of filter_img3_kernel: 1 no appends, 2 no epilogue, 4 no MFMA,
# 8 no query DMA, 16 no step barrier, 32 no image loads), plus ring-depth A/B.
set -o pipefail
mkdir -p gpurun_out
FENIX_AMD_LIB=$PWD/fenix_amd/lib/libfenix_knn_diag.so timeout -k 10 600 python -u tools/filter_diag.py \
  --diags 0,1,2,6,10,14,30,34,18,50,46 > gpurun_out/i3_diag.log 2>&1 || { echo diag failed; tail gpurun_out/i3_diag.log; exit 1; }
cat gpurun_out/i3_diag.log
for rep in 1 2; do
  for v in new qa2 i2; do
    if [ "$v" = new ]; then unset FENIX_AMD_LIB; else export FENIX_AMD_LIB=$PWD/fenix_amd/lib/libfenix_knn_$v.so; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --nq 256 --metric cosine > gpurun_out/i3_b.json 2>gpurun_out/i3_b.err || { echo "bench failed $v"; tail -5 gpurun_out/i3_b.err; exit 1; }
    python -c "import json;r=json.load(open('gpurun_out/i3_b.json'));print('$v', round(r['ms_per_step'],3), round(r['roofline']['kernel_ms'],3))"
  done
done
