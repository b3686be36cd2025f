#!/bin/bash
# int8 filter: image/batched/fallback tests, bench (int8 and fp16), kernel timeline.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "filter_image or batched or single_query_through or overflow or host_sync" > gpurun_out/i8_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/i8_tests.log; exit 1; }
tail -1 gpurun_out/i8_tests.log
for m in cosine l2 inner_product; do
  for b in 8 16; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --nq 256 --metric $m --opt filter_image=$b > gpurun_out/i8_b.json 2>gpurun_out/i8_b.err || { echo "bench failed $m $b"; tail -5 gpurun_out/i8_b.err; exit 1; }
    python -c "import json;r=json.load(open('gpurun_out/i8_b.json'));print('$m bits=$b', round(r['ms_per_step'],3), round(r['roofline']['kernel_ms'],3), r.get('filter_image',{}).get('build_ms'))"
  done
done
bash tools/prof_i8.sh > /dev/null
python tools/timeline.py gpurun_out/prof_i8_trace.csv qprep8 > gpurun_out/prof_i8_timeline.txt
cat gpurun_out/prof_i8_timeline.txt
