#!/bin/bash
# SQ counter pass over one bench configuration (separate from any trace run).
# usage: bash tools/pmc_sq.sh NAME bench-args...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
name=$1
shift
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES -d "gpurun_out/pmc_$name" -o run --output-format csv -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > "gpurun_out/pmc_$name.log" 2>&1
