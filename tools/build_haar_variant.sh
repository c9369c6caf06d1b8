#!/bin/bash
# Build a variant of libffd.so with extra compile flags for the detector (ffd_haar.hip and
# ffd_detect.cpp; the other objects are the default build's).
# usage: tools/build_haar_variant.sh TAG "-DFLAG=1 ..."  -> probe_libs/libffd_TAG.so (tools/detect_ab.sh TAG)
set -eu
cd "$(dirname "$0")/.."
TAG=$1; X=${2:-}
L=face_alignment_cvpr_2012_amd/lib
C=face_alignment_cvpr_2012_amd/csrc
O=probe_libs/obj/$TAG
mkdir -p $O
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Iinclude $X"
/opt/rocm/bin/hipcc $F -c $C/ffd_haar.hip -o $O/ffd_haar.o
/opt/rocm/bin/hipcc $F -c $C/ffd_detect.cpp -o $O/ffd_detect.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o probe_libs/libffd_$TAG.so $L/ffd_kernels.o $L/ffd_engine.o \
  $L/ffd_group.o $L/ffd_archive.o $O/ffd_haar.o $O/ffd_detect.o $L/ffd_train_k.o $L/ffd_train.o -L/opt/rocm/lib -lrccl
echo "probe_libs/libffd_$TAG.so: $X"
