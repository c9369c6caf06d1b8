#!/bin/bash
# PMC groups (tools/pmc_groups_r2.txt or $PMC_GROUPS) over probe builds of the library.
# usage: tools/pmc_builds.sh TAG "EXTRA flags 1" "EXTRA flags 2" ...  -> gpurun_out/pmc_TAG_<i>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
i=0
for x in "$@"; do
  i=$((i+1))
  rm -f face_alignment_cvpr_2012_amd/lib/*.o face_alignment_cvpr_2012_amd/lib/libffd.so
  make -j16 EXTRA="$x" face_alignment_cvpr_2012_amd/lib/libffd.so > gpurun_out/pmc_build.log 2>&1 || exit 3
  echo "build $i: $x" | tee -a gpurun_out/pmc_${TAG}_builds.txt
  PMC_GROUPS=${PMC_GROUPS:-$PWD/tools/pmc_groups_r2.txt} bash tools/pmc.sh ${TAG}_$i || exit $?
done
