#!/bin/bash
# A quick GPU pass: box facts, the named -m gpu test files, then one default
# bench line.  Each GPU step has its own limit; the first failure ends it.
#   bash tools/gpu_first.sh "tests/test_a.py tests/test_b.py" [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/q
export TMPDIR=/tmp
TESTS=$1
shift
{ df -h /tmp . ; free -g ; nproc ; } > gpurun_out/q/box.txt 2>&1
if [ -n "$TESTS" ]; then
  echo "== tests ($(date +%T))"
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/q/tests.log 2>&1
  rc=$?
  echo "   tests rc=$rc"; tail -n 15 gpurun_out/q/tests.log
  [ $rc -eq 0 ] || exit $rc
fi
echo "== bench ($(date +%T))"
timeout -k 10 300 python -u bench.py "$@" > gpurun_out/q/bench.log 2>&1
rc=$?
echo "   bench rc=$rc"; tail -c 3000 gpurun_out/q/bench.log
exit $rc
