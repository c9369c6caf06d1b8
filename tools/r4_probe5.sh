#!/bin/bash
# Round 4: two-walks-per-lane traversal (build/dual) against the in-tree build: leaves on every C2 face and
# 512 C4 faces (far pairs), then the traversal stage times of base / single (DUAL=0) / dual.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=face_alignment_cvpr_2012_amd/lib/libffd.so
ab() {  # workload faces
  FFD_LIBRARY=$PWD/$B timeout -k 10 300 python tools/leaf_ab.py --workload $1 --faces $2 --out gpurun_out/ab_base_$1.npz > gpurun_out/ab_$1.log 2>&1 || { tail -5 gpurun_out/ab_$1.log; exit 1; }
  for v in ${VARIANTS:-dual}; do
    FFD_LIBRARY=$PWD/build/$v/libffd.so timeout -k 10 300 python tools/leaf_ab.py --workload $1 --faces $2 --out gpurun_out/ab_${v}_$1.npz >> gpurun_out/ab_$1.log 2>&1 || { tail -5 gpurun_out/ab_$1.log; exit 1; }
    echo "$v $1: $(python tools/leaf_ab.py --compare gpurun_out/ab_base_$1.npz gpurun_out/ab_${v}_$1.npz)"
  done
}
ab c2 4096
ab c4 512
STAGES=headpose_traverse,ffd_traverse tools/lib_variant_probe.sh $(for v in ${VARIANTS:-dual}; do echo build/$v/libffd.so; done)
