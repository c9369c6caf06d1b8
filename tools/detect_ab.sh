#!/bin/bash
# Detector A/B: the C3 --detect bench's detection time with the default libffd.so and with each
# probe_libs/libffd_TAG.so (FFD_LIBRARY), alternating.  usage: tools/detect_ab.sh TAG [TAG ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for tag in base "$@"; do
    lib=$PWD/probe_libs/libffd_$tag.so
    [ "$tag" = base ] && lib=$PWD/face_alignment_cvpr_2012_amd/lib/libffd.so
    FFD_LIBRARY=$lib timeout -k 10 300 python -u bench.py --workload c3 --detect --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/detab_$tag.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/detab_$tag.log; exit $rc; }
    tail -1 gpurun_out/detab_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['detect'])"
  done
done
