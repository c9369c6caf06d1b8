#!/bin/bash
# Round 5 baseline: the C2 bench line (no CPU baseline / host paths) and one L2 counter pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5
timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-paths > gpurun_out/r5/base_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r5/base_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step'])"
PMC_GROUPS=$PWD/tools/pmc_groups_l2.txt BENCH_ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-host-paths" bash tools/pmc.sh r5_l2 || exit $?
python3 tools/pmc_table.py gpurun_out/pmc_r5_l2 traverse gabor meanshift votes > gpurun_out/r5/l2_table.txt
cat gpurun_out/r5/l2_table.txt
