#!/bin/bash
# Same-box A/B of builds of the library (box-to-box HBM variance is a few per
# cent, larger than most kernel changes).  Build the variants first, e.g.
#   git stash && make -C fenix_amd/csrc BUILD=build_old OUT=../lib/libfenix_knn_old.so && git stash pop
# then: gpurun -- 'LIBS="new old" bash tools/ab_libs.sh [bench.py args...]'
# ("new" is fenix_amd/lib/libfenix_knn.so, NAME is fenix_amd/lib/libfenix_knn_NAME.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
ARGS=${*:-"--nq 256 --metric cosine"}
for i in 1 2; do
  for v in ${LIBS:-new old}; do
    if [ "$v" = new ]; then unset FENIX_AMD_LIB; else export FENIX_AMD_LIB=$PWD/fenix_amd/lib/libfenix_knn_$v.so; fi
    log=gpurun_out/ab_$v.$i.log
    timeout -k 10 200 python -u bench.py $ARGS --steps 10 --warmup 2 --no-cpu-baseline > $log 2>&1 || exit 1
    python -c "
import json
r = json.loads([x for x in open('$log') if x.startswith('{')][-1])
print('$v', $i, round(r['ms_per_step'], 3), round(r['roofline']['kernel_ms'], 3))"
  done
done
