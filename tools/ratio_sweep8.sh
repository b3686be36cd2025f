#!/bin/bash
# Sample-ratio sweep of the int8-image filter phases (option batch_sample_ratio;
# default 8), configs[2] shape: ms per search and the event-timed kernel span.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
 for m in cosine l2; do
  for r in 0 12 16 20 32 40; do
   o=""; [ $r != 0 ] && o="--opt batch_sample_ratio=$r"
   timeout -k 10 300 python -u bench.py --nq 256 --metric $m --steps 10 --warmup 3 --no-cpu-baseline $o \
     > gpurun_out/rs.json 2> gpurun_out/rs.err || { echo "bench failed $m r=$r"; tail -5 gpurun_out/rs.err; exit 1; }
   python -c "import json;r=json.load(open('gpurun_out/rs.json'));print('$m r=$r', round(r['ms_per_step'],3), round(r['roofline']['kernel_ms'],3))"
  done
 done
done
