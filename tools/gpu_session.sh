#!/bin/bash
# One GPU session on the gpurun box: each step has its own time limit; a
# timeout / abort / segfault ends the session (no further GPU step).
# Usage: bash tools/gpu_session.sh STEP...   (steps: smoke tests bench prof pmc)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 secs=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) return 0 ;;
    *) echo "   stopping: $name ended with $rc"; exit "$rc" ;;
  esac
}
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 1200 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider ;;
    testcoder) run pytest_coder 900 python -u -m pytest tests/test_gpu_coder.py -m gpu -q -x -p no:cacheprovider ;;
    coded) run coded 600 python -u tools/bench_coded.py ;;
    profcoded) run profcoded 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profcoded -o run --output-format csv -- python3 -u tools/bench_coded.py --iters 3 ;;
    testq8) run pytest_q8 600 python -u -m pytest tests/test_gpu_quint8.py -m gpu -q -x -p no:cacheprovider ;;
    benchq8) run benchq8 600 python -u bench.py --dtype qu8 --steps 10 --warmup 2 ;;
    benchq8all) run benchq8ip 300 python -u bench.py --dtype qu8 --steps 10 --warmup 2 --metric inner_product --no-cpu-baseline && run benchq8cos 300 python -u bench.py --dtype qu8 --steps 10 --warmup 2 --metric cosine --no-cpu-baseline ;;
    profq8) run profq8 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profq8 -o run --output-format csv -- python3 -u bench.py --dtype qu8 --steps 10 --warmup 2 --no-cpu-baseline ;;
    testbatch) run pytest_batch 900 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k batch -p no:cacheprovider ;;
    bench3l2) run bench3l2 900 python -u bench.py --nq 256 --metric l2 --steps 5 --warmup 1 --no-cpu-baseline ;;
    bench3ip) run bench3ip 900 python -u bench.py --nq 256 --metric inner_product --steps 5 --warmup 1 --no-cpu-baseline ;;
    ktrace3) run ktrace3 600 rocprofv3 --kernel-trace -d gpurun_out/ktrace3 -o run --output-format csv -- python3 -u bench.py --nq 256 --metric cosine --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmcsq3) run pmcsq3 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/pmcsq -o run --output-format csv -- python3 -u bench.py --nq 256 --metric cosine --steps 1 --warmup 0 --no-cpu-baseline ;;
    testk) run pytest_kernels 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -m gpu -q -x -p no:cacheprovider ;;
    testsall) run pytest_gpu 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench) run bench 600 python -u bench.py ;;
    bench3) run bench3 900 python -u bench.py --nq 256 --metric cosine --steps 5 --warmup 1 --no-cpu-baseline ;;
    prof3) run prof3 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python3 -u bench.py --nq 256 --metric cosine --steps 3 --warmup 1 --no-cpu-baseline ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    pmc3) run pmc3 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc3 -o run --output-format csv -- python3 -u bench.py --nq 256 --metric cosine --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmc) run pmc 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o run --output-format csv -- python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
    flight1) run flight1 600 python -u tools/bench_flight.py --n 100000 --d 128 --k 10 --metric l2 ;;
    flight5) run flight5 900 python -u tools/bench_flight.py --n 1000000 --d 1536 --k 1000 --metric inner_product --dtype f16 --reps 10 ;;
    bench5) run bench5 600 python -u bench.py --rows 6250000 --d 1536 --k 1000 --metric inner_product --dtype f16 --steps 10 --warmup 2 --no-cpu-baseline ;;
    prof5) run prof5 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python3 -u bench.py --rows 6250000 --d 1536 --k 1000 --metric inner_product --dtype f16 --steps 10 --warmup 2 --no-cpu-baseline ;;
    microb) run microb 900 python -u tools/microbench.py --nq 256 --metric 2 --occ 0 --rounds 2 --iters 3 ;;
    benchw2) run benchw2 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --rows 2000000 --dist-backend gloo ;;
    micro) run microbench 900 python -u tools/microbench.py --occ 0,2 --groups 0,8,16,32,64 ;;
    sweep) run sweep 900 python -u tools/microbench.py --sweep 128:f32,256:f32,768:f32,1536:f32,768:f16,1536:f16 --occ 0,1,2,3,4 --rounds 2 --iters 6 ;;
    vsweep) run vsweep 1100 python -u tools/microbench.py --variants --sweep 768:f32,128:f32,256:f32,768:f16,1536:f16,1536:f32,100:f32 --occ 0,2 --rounds 2 --iters 5 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done"
