#!/bin/bash
# Round 5 detector A/B: C3 detection time (bench --workload c3 --detect) of the working tree's libffd.so and of saved
# libraries ablib/libffd_TAG.so, alternating, after the detector parity tests on each library.
# usage: tools/r5_c3_ab.sh TAG [TAG ...]   -> gpurun_out/r5/c3ab_*.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5
ARGS="--workload c3 --detect --steps 3 --warmup 1 --no-cpu-baseline --no-host-paths"
for tag in "$@"; do
  FFD_LIBRARY=$PWD/ablib/libffd_$tag.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    -m gpu tests/test_gpu_detect.py -k "not crowded" > gpurun_out/r5/c3ab_tests_$tag.log 2>&1
  rc=$?; echo "$tag tests: $(tail -1 gpurun_out/r5/c3ab_tests_$tag.log)"; [ $rc -eq 0 ] || exit $rc
done
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], 'detect_ms', d['detect']['detect_ms_per_step'])" "$1" "$2"; }
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/r5/c3ab_new.log 2>&1 || exit $?
  summ gpurun_out/r5/c3ab_new.log new
  for tag in "$@"; do
    FFD_LIBRARY=$PWD/ablib/libffd_$tag.so timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/r5/c3ab_$tag.log 2>&1 || exit $?
    summ gpurun_out/r5/c3ab_$tag.log $tag
  done
done
