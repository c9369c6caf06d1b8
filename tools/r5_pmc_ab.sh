#!/bin/bash
# PMC passes (tools/pmc_groups_tatd.txt) on the working tree's libffd.so and on saved libraries (ablib/libffd_TAG.so).
# usage: tools/r5_pmc_ab.sh TAG...   -> gpurun_out/pmc_r5_new, gpurun_out/pmc_r5_TAG, gpurun_out/r5/pmc_*.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5
export PMC_GROUPS=$PWD/tools/pmc_groups_tatd.txt BENCH_ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-host-paths"
bash tools/pmc.sh r5_new || exit $?
python3 tools/pmc_table.py gpurun_out/pmc_r5_new traverse > gpurun_out/r5/pmc_new.txt
for tag in "$@"; do
  FFD_LIBRARY=$PWD/ablib/libffd_$tag.so bash tools/pmc.sh r5_$tag || exit $?
  python3 tools/pmc_table.py gpurun_out/pmc_r5_$tag traverse > gpurun_out/r5/pmc_$tag.txt
done
