#!/bin/bash
# A libffd.so whose Haar kernels (ffd_haar.hip) get extra compile flags, the other objects the default build's.
# usage: tools/build_haar_variant.sh NAME "-DFLAG=1 ..."  -> ablib/libffd_NAME.so (travels to the GPU box)
set -eu
cd "$(dirname "$0")/.."
NAME=$1; X=${2:-}
L=face_alignment_cvpr_2012_amd/lib
mkdir -p ablib /tmp/hv_$NAME
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
  -Iinclude $X -c face_alignment_cvpr_2012_amd/csrc/ffd_haar.hip -o /tmp/hv_$NAME/ffd_haar.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ablib/libffd_$NAME.so $L/ffd_kernels.o $L/ffd_engine.o \
  $L/ffd_group.o $L/ffd_archive.o /tmp/hv_$NAME/ffd_haar.o $L/ffd_detect.o $L/ffd_train_k.o $L/ffd_train.o \
  $L/ffd_convert.o -L/opt/rocm/lib -lrccl
echo "ablib/libffd_$NAME.so: $X"
