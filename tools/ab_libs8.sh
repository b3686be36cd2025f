#!/bin/bash
# Same-box A/B of library variants on configs[2] (10M x 768 f32, 256 queries,
# k = 100) through the int8 filter image: ms per search and the event-timed
# kernel span.  Usage: tools/ab_libs8.sh "VARIANT..." "METRIC..." [REPS] [-- bench options]
# (variant "new" = the product library, else fenix_amd/lib/libfenix_knn_<v>.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
vars=$1; mets=$2; reps=${3:-2}; shift 3; [ "$1" = "--" ] && shift
for rep in $(seq $reps); do
  for v in $vars; do
    if [ "$v" = new ]; then unset FENIX_AMD_LIB; else export FENIX_AMD_LIB=$PWD/fenix_amd/lib/libfenix_knn_$v.so; fi
    for m in $mets; do
      timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --nq 256 --metric $m "$@" \
        > gpurun_out/ab8.json 2>gpurun_out/ab8.err || { echo "bench failed $v $m"; tail -5 gpurun_out/ab8.err; exit 1; }
      python -c "import json;r=json.load(open('gpurun_out/ab8.json'));print('$v $m $*', round(r['ms_per_step'],3), round(r['roofline']['kernel_ms'],3))"
    done
  done
done
unset FENIX_AMD_LIB
