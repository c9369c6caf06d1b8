#!/bin/bash
# L2 hit/miss counters for the traversal in its three probe modes (combined, walk only, stage only).
# usage: tools/pmc_l2.sh TAG   -> gpurun_out/pmc_l2_TAG/<mode>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/pmc_l2_${1:-l2}
mkdir -p "$OUT"
for mode in 0 2 1; do
  rm -f face_alignment_cvpr_2012_amd/lib/*.o face_alignment_cvpr_2012_amd/lib/libffd.so
  make -j16 EXTRA="-DFFD_TRAV_PROBE=$mode" face_alignment_cvpr_2012_amd/lib/libffd.so > "$OUT/build.log" 2>&1 || exit 3
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/m$mode" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/m$mode.log" 2>&1)
  rc=$?; echo "mode $mode rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
