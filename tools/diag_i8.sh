#!/bin/bash
# Diagnostic matrix of the int8 filter (diagnostic build, results not
# checked): FX_FILTER_DIAG bits 1 no appends, 2 no epilogue, 4 no MFMA,
# 8 no query DMA, 16 no step barrier, 32 no image loads; configs[2] cosine.
set -o pipefail
mkdir -p gpurun_out
export FENIX_AMD_LIB=$PWD/fenix_amd/lib/libfenix_knn_diag.so
for rep in 1 2; do
  for dg in 0 1 2 6 10 34 14 42 38 46; do
    FX_FILTER_DIAG=$dg timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-verify --nq 256 --metric cosine > gpurun_out/d8_b.json 2>gpurun_out/d8_b.err || { echo "bench failed $dg"; tail -5 gpurun_out/d8_b.err; exit 1; }
    python -c "import json;r=json.load(open('gpurun_out/d8_b.json'));print('diag=$dg', round(r['ms_per_step'],3), round(r['roofline']['kernel_ms'],3))"
  done
done
