#!/bin/bash
# Round 6: filter_img9_kernel (option img8=2) against filter_img8_kernel:
# parity test, repeat check, configs[2] timing with a kernel trace per variant.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06/img9
mkdir -p $O
run() {
  local name=$1 secs=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   $name rc=$rc"
  tail -n 3 "$O/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
run parity 400 python -u -m pytest tests/test_gpu_kernels.py -k "img8_queries_in_registers" -x -v --timeout 300 --timeout-method thread
run race 300 python -u tools/race_check.py --reps 12 --nq 129,256,300 --d 136,768 --n 600000 --img6 1 --img8 1,2 --metric 2
for v in 1 2 1 2; do
  run "bench_img8_$v" 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 -u bench.py --nq 256 --metric cosine --steps 20 --warmup 3 --no-cpu-baseline --opt img8=$v
  grep -h '^{' $O/bench_img8_$v.log >> $O/bench_lines.jsonl
  python3 tools/ktrace_summary.py $O/prof_$v/run_kernel_trace.csv >> $O/ktrace_$v.txt 2>&1 || true
done
echo "== done"
