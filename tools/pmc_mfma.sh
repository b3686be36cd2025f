#!/bin/bash
# MFMA/LDS counter pass over the batched cosine bench (configs[2]).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/pmc_mfma -o run --output-format csv -- python3 -u bench.py --nq 256 --metric cosine --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_mfma.log 2>&1
