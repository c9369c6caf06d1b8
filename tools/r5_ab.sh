#!/bin/bash
# Round 5 A/B: GPU parity tests of the traversal on the working tree's libffd.so, then the C2 bench
# alternating between the working tree's build and saved libraries (ablib/libffd_TAG.so).
# usage: tools/r5_ab.sh "TESTS" TAG [TAG ...]     (TESTS="" skips the tests)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5
TESTS=$1; shift
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/r5/ab_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/r5/ab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], 'hp', s['headpose_traverse'], 'ffd', s['ffd_traverse'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), 'ms', s['meanshift'], 'votes', s['votes'])" "$1" "$2"; }
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-host-paths > gpurun_out/r5/ab_new.log 2>&1 || exit $?
  summ gpurun_out/r5/ab_new.log new
  for tag in "$@"; do
    FFD_LIBRARY=$PWD/ablib/libffd_$tag.so timeout -k 10 300 python3 bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-host-paths > gpurun_out/r5/ab_$tag.log 2>&1 || exit $?
    summ gpurun_out/r5/ab_$tag.log $tag
  done
done
