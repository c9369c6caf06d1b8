#!/bin/bash
# Round 4 end-of-round evidence in one call: pytest -m gpu, smoke(), tools/profile_round.sh TAG (rocprofv3
# kernel-trace summary, FETCH_SIZE / WRITE_SIZE passes -> traffic.json, the bench line with its CPU baseline),
# then the C3 (--detect), C4 and C5 bench lines.  -> gpurun_out/round_TAG/, gpurun_out/configs_TAG/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r4b}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gt_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/gt_$TAG.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/gt_$TAG.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
bash tools/profile_round.sh $TAG || exit $?
WORKLOADS="c3 c4 c5" BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-host-paths" bash tools/bench_configs.sh $TAG
