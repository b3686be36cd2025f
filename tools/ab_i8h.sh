#!/bin/bash
# Timing bound for an int8-MFMA filter (diagnostic builds, results not
# checked): the fp16 img3 kernel vs the same kernel with int8 MFMA over
# 64-component chunks (FX_I3_I8, half the image bytes), configs[2] shapes,
# without appends (FX_FILTER_DIAG=1) and without the epilogue (2).
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in diag i8h; do
    export FENIX_AMD_LIB=$PWD/fenix_amd/lib/libfenix_knn_$v.so
    for dg in 1 2 3; do
      FX_FILTER_DIAG=$dg timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-verify --nq 256 --metric cosine > gpurun_out/i8h_b.json 2>gpurun_out/i8h_b.err || { echo "bench failed $v"; tail -5 gpurun_out/i8h_b.err; exit 1; }
      python -c "import json;r=json.load(open('gpurun_out/i8h_b.json'));print('$v diag=$dg', round(r['ms_per_step'],3), round(r['roofline']['kernel_ms'],3))"
    done
  done
done
