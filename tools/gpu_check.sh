#!/bin/bash
# One gpurun call: GPU parity tests, then a short bench, then a rocprofv3 kernel-trace summary.
# Stops at the first step that crashes / times out (exit status other than 0 or 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r1}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 ${TEST_TIMEOUT:-420} python -m pytest tests -x -q -m gpu ${PYTEST_ARGS:-} > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/tests_$TAG.log; tail -5 gpurun_out/tests_$TAG.log
ok $rc || exit $rc
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
timeout -k 10 ${BENCH_TIMEOUT:-420} python bench.py ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/bench_$TAG.log; tail -3 gpurun_out/bench_$TAG.log
[ $rc -eq 0 ] || exit $rc
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${PROF_TIMEOUT:-420} rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc" | tee -a "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log"
exit $rc
