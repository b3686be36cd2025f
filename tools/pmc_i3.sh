#!/bin/bash
# SQ counter pass over configs[2] (img3 product build), then FETCH_SIZE.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_i3sq -o run --output-format csv -- python3 -u bench.py --nq 256 --metric cosine --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_i3sq.log 2>&1 || { echo "sq pass failed"; tail -5 gpurun_out/pmc_i3sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/pmc_i3sq2 -o run --output-format csv -- python3 -u bench.py --nq 256 --metric cosine --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_i3sq2.log 2>&1 || { echo "sq2 pass failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_i3 -o run --output-format csv -- python3 -u bench.py --nq 256 --metric cosine --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/kt_i3.log 2>&1 || { echo "kt failed"; exit 1; }
find gpurun_out/pmc_i3sq gpurun_out/pmc_i3sq2 gpurun_out/kt_i3 -name "*.csv" | head
