#!/bin/bash
# Round-6 measurement steps on one GPU box, chosen by name:
#   bash tools/r06_job.sh bench flightprof flight k1000 ...
# bench      default bench.py line (configs[1] headline + legs)
# flightprof io.index.call phase breakdown + cProfile at configs[1]'s shape
# flight     Flight.search from a torch-free client at configs[1]'s shape
# k1000      one configs[4] shard (6.25M x 1536 f16 IP k=1000): exact scan vs
#            the int8 image with i8_max_k raised (candidate counts, time)
# Each GPU step has its own limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
run() {
  local name=$1 secs=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/r06/$name.log" 2>&1
  local rc=$?
  echo "   $name rc=$rc"
  tail -n 4 "gpurun_out/r06/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
TESTS=${TESTS:-tests}
K4="--dtype f16 --d 1536 --rows 6250000 --k 1000 --metric inner_product --no-batch-leg --opt i8_max_k=1024"
for step in "$@"; do
  case $step in
    bench) run bench 300 python -u bench.py ;;
    flightprof) run flightprof 600 python -u tools/profile_call.py --n 10000000 --d 768 --dtype f32 \
        --metric l2 --k 100 --batch 1000 --reps 30 --json gpurun_out/r06/flightprof.json ;;
    flight) run flight 600 python -u tools/bench_flight.py --n 10000000 --d 768 --k 100 --metric l2 \
        --direct --reps 60 ;;
    flightc) run flightc 600 python -u tools/bench_flight.py --n 10000000 --d 768 --k 100 --metric l2 \
        --direct --reps 60 --canned ;;
    tests) run tests 900 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 \
        --timeout-method thread ;;
    ksweep) run ksweep 900 python -u tools/k1000_sweep.py --queries 20 --opt i8_max_k=1024 \
        --json gpurun_out/r06/k1000_sweep.json ;;
    ktrace) run ktrace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/ktrace -o run \
        --output-format csv -- python3 -u bench.py --dtype f16 --d 1536 --rows 6250000 --k 1000 \
        --metric inner_product --no-cpu-baseline --no-batch-leg --opt i8_max_k=1024 --steps 5 --warmup 1
      python tools/timeline.py gpurun_out/r06/ktrace/run_kernel_trace.csv qprep8 \
        > gpurun_out/r06/ktrace_timeline.txt ;;
    ctrace) run ctrace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/ctrace -o run \
        --output-format csv -- python3 -u bench.py --no-cpu-baseline --no-batch-leg --steps 5 --warmup 1
      python tools/timeline.py gpurun_out/r06/ctrace/run_kernel_trace.csv qprep8 \
        > gpurun_out/r06/ctrace_timeline.txt ;;
    flightr) run flightr 600 python -u tools/bench_flight.py --n 10000000 --d 768 --k 100 --metric l2 \
        --direct --reps 60 --read-all ;;
    rsweep1) run rsweep1 900 python -u tools/sweep.py --reps 2 --steps 20 --warmup 3 \
        --out gpurun_out/r06/ratio_sweep_cfg1.jsonl -- "--no-batch-leg" \
        "--no-batch-leg --opt i8_grow_ratio=32 --opt select_prune=2" \
        "--no-batch-leg --opt i8_grow_ratio=20 --opt select_prune=2" \
        "--no-batch-leg --opt select_prune=2" "--no-batch-leg --opt i8_sample_ratio=12" ;;
    rsweep4) run rsweep4 900 python -u tools/sweep.py --reps 1 --steps 20 --warmup 3 \
        --out gpurun_out/r06/ratio_sweep_k1000.jsonl -- \
        "$K4 --opt i8_grow_ratio=16" "$K4 --opt i8_grow_ratio=8" "$K4 --opt i8_grow_ratio=32" \
        "$K4 --opt i8_sample_ratio=4" "$K4 --opt i8_sample_ratio=16" "$K4 --opt select_prune=0" ;;
    kbatch) K16="--dtype f16 --d 1536 --rows 6250000 --metric inner_product --no-batch-leg --k 1000"
      run kbatch 1100 python -u tools/sweep.py --reps 1 --steps 10 --warmup 2 \
        --out gpurun_out/r06/kbatch.jsonl -- \
        "$K16 --nq 16 --opt i8_max_k=256" "$K16 --nq 16 --opt i8_max_k=1024" \
        "$K16 --nq 256 --opt i8_max_k=256" "$K16 --nq 256 --opt i8_max_k=1024" \
        "--no-batch-leg --k 1000 --nq 16 --opt i8_max_k=256" "--no-batch-leg --k 1000 --nq 16 --opt i8_max_k=1024" \
        "--no-batch-leg --k 300 --nq 256 --metric cosine --opt i8_max_k=256" \
        "--no-batch-leg --k 300 --nq 256 --metric cosine --opt i8_max_k=1024" ;;
    kclust) run kclust 900 python -u tools/k1000_sweep.py --queries 10 --cluster 1000 --opt i8_max_k=1024 \
        --json gpurun_out/r06/k1000_sweep_cluster.json ;;
    abseg) run abseg 1100 python -u tools/sweep.py --libs new,old --reps 2 --steps 20 --warmup 3 \
        --out gpurun_out/r06/abseg.jsonl -- "--no-batch-leg" "--no-batch-leg --nq 256 --metric cosine" \
        "$K4" ;;
    rtrace) run rtrace 300 rocprofv3 --runtime-trace --kernel-trace --memory-copy-trace -d gpurun_out/r06/rtrace \
        -o run --output-format csv -- python3 -u tools/profile_call.py --n 10000000 --d 768 --dtype f32 \
        --metric l2 --k 100 --batch 1000 --reps 30
      python tools/host_gap.py gpurun_out/r06/rtrace/run > gpurun_out/r06/rtrace_gap.txt 2>&1 ;;
    sq) run sq1 200 bash tools/pmc.sh img8_sq1 "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" \
        --nq 256 --metric cosine --no-verify --no-accelerated
      run sq2 200 bash tools/pmc.sh img8_sq2 "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES" \
        --nq 256 --metric cosine --no-verify --no-accelerated
      python tools/sq_summary.py gpurun_out/pmc_img8_sq1/run_counter_collection.csv filter_img8 > gpurun_out/r06/sq_img8.txt
      python tools/sq_summary.py gpurun_out/pmc_img8_sq2/run_counter_collection.csv filter_img8 >> gpurun_out/r06/sq_img8.txt ;;
    cfg4test) run cfg4test 600 python -u -m pytest tests/test_gpu_sharded.py -m gpu -x -v -p no:cacheprovider \
        --timeout 500 --timeout-method thread -k configs4 ;;
    flight4) run flight4 600 python -u tools/bench_flight.py --n 6250000 --d 1536 --k 1000 --metric inner_product \
        --dtype f16 --direct --reps 40 ;;
    gsweep) run gsweep 1100 python -u tools/sweep.py --reps 2 --steps 20 --warmup 3 \
        --out gpurun_out/r06/grow_sweep.jsonl -- "--no-batch-leg" "--no-batch-leg --opt i8_grow_ratio=32" \
        "--no-batch-leg --opt i8_grow_ratio=64" "--no-batch-leg --opt i8_grow_ratio=128" \
        "--no-batch-leg --opt i8_grow_ratio=64 --opt select_prune=2" \
        "--no-batch-leg --nq 256 --metric cosine" "--no-batch-leg --nq 256 --metric cosine --opt i8_grow_ratio=64" ;;
    ctrace2) run ctrace2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/ctrace2 -o run \
        --output-format csv -- python3 -u bench.py --nq 256 --metric cosine --no-cpu-baseline --steps 5 --warmup 1
      python tools/timeline.py gpurun_out/r06/ctrace2/run_kernel_trace.csv qprep8 \
        > gpurun_out/r06/ctrace2_timeline.txt ;;
    rsweep2) C2="--no-batch-leg --nq 256 --metric cosine"
      run rsweep2 1100 python -u tools/sweep.py --reps 2 --steps 20 --warmup 3 \
        --out gpurun_out/r06/ratio_sweep_cfg2.jsonl -- "$C2" "$C2 --opt i8_grow_ratio=8" \
        "$C2 --opt i8_grow_ratio=12" "$C2 --opt i8_sample_ratio=6" "$C2 --opt i8_sample_ratio=10" \
        "$C2 --opt i8_sample_ratio=12" "--no-batch-leg --opt i8_grow_ratio=8" \
        "--no-batch-leg --opt i8_sample_ratio=6" "--no-batch-leg --opt i8_sample_ratio=10" ;;
    rsweep3) run rsweep3 1100 python -u tools/sweep.py --reps 3 --steps 30 --warmup 3 \
        --out gpurun_out/r06/ratio_sweep_s6.jsonl -- "--no-batch-leg" "--no-batch-leg --opt i8_sample_ratio=6" \
        "--no-batch-leg --opt i8_sample_ratio=5" "--no-batch-leg --opt i8_sample_ratio=7" \
        "$K4" "$K4 --opt i8_sample_ratio=6" ;;
    flight0) run flight0 300 python -u tools/bench_flight.py --n 100000 --d 128 --k 10 --metric l2 --reps 60 ;;
    k1000) run k1000a 300 python -u bench.py --dtype f16 --d 1536 --rows 6250000 --k 1000 \
        --metric inner_product --no-cpu-baseline --no-batch-leg --opt i8_max_k=1024
      run k1000b 300 python -u bench.py --dtype f16 --d 1536 --rows 6250000 --k 1000 \
        --metric inner_product --no-cpu-baseline --no-batch-leg --opt i8_max_k=1024 --query near ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done"
