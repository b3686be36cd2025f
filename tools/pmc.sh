#!/bin/bash
# One rocprofv3 counter pass over one bench.py configuration (its own run:
# never combined with a trace; at most 8 SQ / 4 TCC counters per pass).
#   bash tools/pmc.sh NAME "SQ_WAVE_CYCLES SQ_WAIT_ANY ..." [bench.py args...]
# -> gpurun_out/pmc_NAME/run_counter_collection.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
name=$1
counters=$2
shift 2
mkdir -p gpurun_out
timeout -k 10 -s KILL 300 rocprofv3 --pmc $counters -d "gpurun_out/pmc_$name" -o run --output-format csv -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > "gpurun_out/pmc_$name.log" 2>&1
