#!/bin/bash
# Round 4: k_meanshift4 with one chain per wave (build/msc1: launch4 allowed down to C = 1) at C4, where
# 2 chains per wave beat 4 (FFD_MS_WAVES 16,384 -> C = 1 for C4's 10,240 chains; the default stays C = 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local tag=$1 lib=$2; shift 2
  env FFD_LIBRARY=$lib "$@" timeout -k 10 300 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-host-paths > gpurun_out/msc1_$tag.log 2>&1 || { tail -5 gpurun_out/msc1_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/msc1_$tag.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(d['value'], 'ms', d['stage_ms_per_step']['meanshift'], 'spot', d['landmark_px_error']['faces_identical'], '/', d['landmark_px_error']['faces_checked'])")"
}
B=$PWD/face_alignment_cvpr_2012_amd/lib/libffd.so V=$PWD/build/msc1/libffd.so
run base $B
run c1 $V FFD_MS_WAVES=16384
run base2 $B
run c1b $V FFD_MS_WAVES=16384
