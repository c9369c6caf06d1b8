#!/bin/bash
# Bench the default build against variant builds of libffd.so (FFD_LIBRARY); prints value, the
# bench's parity spot check and the stages named by STAGES (comma-separated) for each.
# usage: STAGES=ffd_traverse,meanshift tools/lib_variant_probe.sh build/a/libffd.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in face_alignment_cvpr_2012_amd/lib/libffd.so "$@"; do
  FFD_LIBRARY=$PWD/$lib timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/bench_variant.log 2>&1 || exit 1
  echo "$lib $(tail -1 gpurun_out/bench_variant.log | python3 -c "
import json, sys, os
d = json.loads(sys.stdin.read())
st = os.environ.get('STAGES', os.environ.get('STAGE', 'meanshift')).split(',')
print(d['value'], 'spot', d.get('landmark_px_error',{}).get('faces_identical'), ' '.join('%s=%s' % (s, d['stage_ms_per_step'].get(s)) for s in st))")" | tee -a gpurun_out/variants.txt
done
