#!/bin/bash
# Bench the default build against variant builds of libffd.so (FFD_LIBRARY); prints value and the
# stage named by STAGE for each.  usage: STAGE=meanshift tools/lib_variant_probe.sh build/a/libffd.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in face_alignment_cvpr_2012_amd/lib/libffd.so "$@"; do
  FFD_LIBRARY=$PWD/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/bench_variant.log 2>&1 || exit 1
  echo "$lib $(tail -1 gpurun_out/bench_variant.log | python3 -c "import json,sys,os; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_per_step'][os.environ.get('STAGE','meanshift')])")"
done
