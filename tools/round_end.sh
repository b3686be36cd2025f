#!/bin/bash
# Round-end evidence on one GPU box: the full -m gpu suite and smoke, the
# configs[1] and configs[2] bench lines, rocprofv3 kernel stats, and
# FETCH_SIZE passes summarised into profiles/rNN_pmc_*.json stamped with the
# library's SHA (copied to gpurun_out/ so they come back), then the bench
# lines again with the traffic fields filled in.  Every GPU step has its own
# limit; a crash, abort or timeout ends the script.
#   bash tools/round_end.sh ROUND [--no-tests | --tests-only]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$(printf "%02d" "${1:-4}")
mkdir -p gpurun_out/re
export TMPDIR=/tmp
run() {
  local name=$1 secs=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/re/$name.log" 2>&1
  local rc=$?
  echo "   $name rc=$rc"
  tail -n 3 "gpurun_out/re/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
CFG2="--nq 256 --metric cosine"
if [ "$2" != "--no-tests" ]; then
  run tests 1300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
  run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
[ "$2" == "--tests-only" ] && { echo "== done"; exit 0; }
run bench1 300 python -u bench.py
run bench2 300 python -u bench.py $CFG2 --no-cpu-baseline
# the headline's kernel alone (exact fused scan; no filter-image leg, whose
# gated fallback would add ~5 us scan_kernel launches to the average)
run prof1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/re/prof1 -o run --output-format csv -- python3 -u bench.py --no-accelerated --steps 10 --warmup 2 --no-cpu-baseline
run prof1a 300 rocprofv3 --kernel-trace --stats -d gpurun_out/re/prof1a -o run --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-batch-leg
run prof2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/re/prof2 -o run --output-format csv -- python3 -u bench.py $CFG2 --steps 5 --warmup 2 --no-cpu-baseline
run pmc1 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/re/pmc1 -o run --output-format csv -- python3 -u bench.py --no-accelerated --steps 5 --warmup 1 --no-cpu-baseline
run pmc1a 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/re/pmc1a -o run --output-format csv -- python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-batch-leg
run pmc2 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/re/pmc2 -o run --output-format csv -- python3 -u bench.py $CFG2 --steps 2 --warmup 1 --no-cpu-baseline
W1=10000000x768_f32_l2_k100_q1
python tools/summarize_profiles.py --round "$R" --stats gpurun_out/re/prof1/run_kernel_stats.csv \
  --pmc gpurun_out/re/pmc1/run_counter_collection.csv --workload $W1 \
  --kernel scan_kernel --algo-bytes 30720003072 \
  --source-cmd "rocprofv3 --pmc FETCH_SIZE -- python3 bench.py --no-accelerated --steps 5 --warmup 1" || exit 1
# the accelerated leg: 6 searches (1 warmup + 5 steps), every filter phase summed
python tools/summarize_profiles.py --round "$R" --tag _img8 --stats gpurun_out/re/prof1a/run_kernel_stats.csv \
  --pmc gpurun_out/re/pmc1a/run_counter_collection.csv --workload $W1 \
  --kernel filter_img --searches 6 --algo-bytes 7840003072 \
  --source-cmd "rocprofv3 --pmc FETCH_SIZE -- python3 bench.py --steps 5 --warmup 1 --no-batch-leg" || exit 1
python tools/summarize_profiles.py --round "$R" --tag _cfg2 --stats gpurun_out/re/prof2/run_kernel_stats.csv \
  --pmc gpurun_out/re/pmc2/run_counter_collection.csv --workload 10000000x768_f32_cosine_k100_q256 \
  --kernel filter_img --searches 3 --algo-bytes 7840786432 \
  --source-cmd "rocprofv3 --pmc FETCH_SIZE -- python3 bench.py $CFG2 --steps 2 --warmup 1" || exit 1
cp profiles/r${R}_* gpurun_out/re/ 2>/dev/null
run bench1t 300 python -u bench.py
run bench2t 300 python -u bench.py $CFG2 --no-cpu-baseline
echo "== done"
