#!/bin/bash
# Build probe / variant copies of libffd.so HERE (CPU container) so a GPU call only runs them:
#   tools/build_variants.sh TAG "EXTRA flags" [TAG "EXTRA flags" ...]  -> probe_libs/libffd_TAG.so
# (ffd_kernels.hip recompiled with the flags, linked with the other objects of the current build).
set -eu
cd "$(dirname "$0")/.."
make -s -j8 face_alignment_cvpr_2012_amd/lib/libffd.so
mkdir -p probe_libs/obj
L=face_alignment_cvpr_2012_amd/lib
OTHERS=$(ls $L/*.o | grep -v ffd_kernels.o)
pids=()
while [ $# -ge 2 ]; do
  tag=$1; flags=$2; shift 2
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude $flags \
      -c face_alignment_cvpr_2012_amd/csrc/ffd_kernels.hip -o probe_libs/obj/ffd_kernels_$tag.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o probe_libs/libffd_$tag.so probe_libs/obj/ffd_kernels_$tag.o $OTHERS \
      -L/opt/rocm/lib -lrccl && echo "built $tag" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
