#!/bin/bash
# Build a variant of libffd.so with extra compile flags for the kernels (the other objects are the
# default build's).  usage: tools/build_variant.sh NAME "-DFLAG=1 ..."  -> build/NAME/libffd.so
# (then on the GPU: tools/lib_variant_probe.sh build/NAME/libffd.so ...)
set -eu
cd "$(dirname "$0")/.."
NAME=$1; X=${2:-}
L=face_alignment_cvpr_2012_amd/lib
mkdir -p build/$NAME
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
  -Iinclude $X -c face_alignment_cvpr_2012_amd/csrc/ffd_kernels.hip -o build/$NAME/ffd_kernels.o
ENG=$L/ffd_engine.o
if [ "${ENGINE:-0}" = 1 ]; then  # flags that change the host-side encodings too (e.g. the record layout)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
    -Iinclude $X -c face_alignment_cvpr_2012_amd/csrc/ffd_engine.cpp -o build/$NAME/ffd_engine.o
  ENG=build/$NAME/ffd_engine.o
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/$NAME/libffd.so build/$NAME/ffd_kernels.o \
  $ENG $L/ffd_group.o $L/ffd_archive.o $L/ffd_haar.o $L/ffd_detect.o $L/ffd_train_k.o $L/ffd_train.o $L/ffd_convert.o -L/opt/rocm/lib -lrccl
echo "build/$NAME/libffd.so: $X"
