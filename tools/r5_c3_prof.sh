#!/bin/bash
# C3 detector profile (round 5): kernel stats of `bench.py --workload c3 --detect`, then SQ counter passes
# (tools/pmc_groups_tatd.txt's two SQ groups) summarised for the Haar kernels.  -> gpurun_out/r5/c3_*
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r5
ARGS="--workload c3 --detect --steps 2 --warmup 1 --no-cpu-baseline --no-host-paths"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5/c3_trace" -o run \
    --output-format csv -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/r5/c3_trace.log" 2>&1 ) || exit $?
grep -v "^TA_\|^TCC" tools/pmc_groups_tatd.txt > /tmp/c3_groups.txt
export PMC_GROUPS=/tmp/c3_groups.txt BENCH_ARGS="$ARGS"
bash tools/pmc.sh r5_c3 || exit $?
python3 tools/pmc_table.py gpurun_out/pmc_r5_c3 haar > gpurun_out/r5/c3_pmc.txt
