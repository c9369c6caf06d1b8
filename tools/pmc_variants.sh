#!/bin/bash
# PMC passes (tools/pmc.sh) for the default libffd.so and each variant library given.
# usage: PMC_GROUPS=tools/pmc_groups_walk.txt tools/pmc_variants.sh TAG build/a/libffd.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
R=$PWD
for lib in face_alignment_cvpr_2012_amd/lib/libffd.so "$@"; do
  name=$(basename "$(dirname "$lib")")
  FFD_LIBRARY=$R/$lib bash tools/pmc.sh "${TAG}_$name" || exit $?
  python3 tools/pmc_table.py "gpurun_out/pmc_${TAG}_$name" k_traverse > "gpurun_out/pmc_${TAG}_$name.txt"
done
