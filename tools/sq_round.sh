#!/bin/bash
# SQ counter evidence for a round in one gpurun call: the GPU parity tests of the channel path, then
# tools/pmc.sh with tools/pmc_groups_sq.txt (2 passes) over the C2 bench and over the C3 --detect bench.
# usage: tools/sq_round.sh TAG  -> gpurun_out/pmc_TAG_c2, gpurun_out/pmc_TAG_c3 (tools/pmc_derived.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-sq}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
PMC_GROUPS=$PWD/tools/pmc_groups_sq.txt BENCH_ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-host-paths" \
  bash tools/pmc.sh ${TAG}_c2 || exit $?
PMC_GROUPS=$PWD/tools/pmc_groups_sq.txt BENCH_ARGS="--workload c3 --detect --steps 1 --warmup 1 --no-cpu-baseline" \
  bash tools/pmc.sh ${TAG}_c3
