#!/bin/bash
# Batched-search times on one box (bench.py, 10Mx768 f32 k=100, filter image
# on): ms per step and kernel ms per batch size / metric.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
run() {
  env "$@" > /dev/null
  timeout -k 10 200 env $ENVS python -u bench.py $ARGS --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bs.log 2>&1 || exit 1
  python -c "
import json
r = json.loads([x for x in open('gpurun_out/bs.log') if x.startswith('{')][-1])
print('$ENVS', '$ARGS', round(r['ms_per_step'], 3), round(r['roofline']['kernel_ms'], 3))"
}
for a in "--nq 1 --metric l2" "--nq 2 --metric l2" "--nq 16 --metric l2" "--nq 64 --metric l2" "--nq 65 --metric l2" "--nq 128 --metric l2" "--nq 256 --metric l2" "--nq 256 --metric inner_product" "--nq 256 --metric cosine"; do
  ENVS=FX_NONE=1 ARGS="$a" run
done
ENVS=FX_BATCH_MIN=1 ARGS="--nq 1 --metric l2" run
