#!/bin/bash
# Round 4: head-pose 4 x 5 blocks (pitch 44: patch rows 2-way instead of 4-way on the LDS banks) in build/hp45
# (FFD_TRAV_G_HP=4x5) against the in-tree 5 x 4: leaves on every C2 face, stage times; then the evaluateMT trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=face_alignment_cvpr_2012_amd/lib/libffd.so
FFD_LIBRARY=$PWD/$B timeout -k 10 300 python tools/leaf_ab.py --faces 4096 --out gpurun_out/ab_base_c2.npz > gpurun_out/ab9.log 2>&1 || { tail -5 gpurun_out/ab9.log; exit 1; }
FFD_TRAV_G_HP=4x5 FFD_LIBRARY=$PWD/build/hp45/libffd.so timeout -k 10 300 python tools/leaf_ab.py --faces 4096 --out gpurun_out/ab_hp45_c2.npz >> gpurun_out/ab9.log 2>&1 || { tail -5 gpurun_out/ab9.log; exit 1; }
echo "hp45 c2: $(python tools/leaf_ab.py --compare gpurun_out/ab_base_c2.npz gpurun_out/ab_hp45_c2.npz)"
STAGES=headpose_traverse,ffd_traverse tools/lib_variant_probe.sh || exit 1
FFD_TRAV_G_HP=4x5 STAGES=headpose_traverse,ffd_traverse tools/lib_variant_probe.sh build/hp45/libffd.so || exit 1
tools/evaluate_mt_trace.sh
