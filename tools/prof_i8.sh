#!/bin/bash
# Kernel-level breakdown of one configs[2] search through the int8 image.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_i8 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --nq 256 --metric cosine > gpurun_out/prof_i8.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_i8.log; exit 1; }
find gpurun_out/prof_i8 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof_i8_stats.csv
find gpurun_out/prof_i8 -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} gpurun_out/prof_i8_trace.csv
head -30 gpurun_out/prof_i8_stats.csv | cut -d, -f1-8
