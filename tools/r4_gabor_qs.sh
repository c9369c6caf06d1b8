#!/bin/bash
# Round 4: Gabor plane-half passes for 13x13 (build/qs13) and 13x13 + 19x19 (build/qs7) against the in-tree build
# (9x9 only): leaves and landmarks on every C2 face, Gabor stage times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=face_alignment_cvpr_2012_amd/lib/libffd.so
FFD_LIBRARY=$PWD/$B timeout -k 10 300 python tools/leaf_ab.py --faces 4096 --out gpurun_out/ab_base_c2.npz > gpurun_out/abq.log 2>&1 || { tail -5 gpurun_out/abq.log; exit 1; }
for v in qs13 qs7 noblk; do
  FFD_LIBRARY=$PWD/build/$v/libffd.so timeout -k 10 300 python tools/leaf_ab.py --faces 4096 --out gpurun_out/ab_${v}_c2.npz >> gpurun_out/abq.log 2>&1 || { tail -5 gpurun_out/abq.log; exit 1; }
  echo "$v c2: $(python tools/leaf_ab.py --compare gpurun_out/ab_base_c2.npz gpurun_out/ab_${v}_c2.npz)"
done
STAGES=gabor_19x19,gabor_13x13,gabor_9x9,headpose_traverse,ffd_traverse tools/lib_variant_probe.sh build/qs13/libffd.so build/qs7/libffd.so build/noblk/libffd.so
