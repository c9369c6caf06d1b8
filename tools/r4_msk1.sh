#!/bin/bash
# Round 4: k_meanshift4 with 1 / 2 votes per lane per tile at C4 (two runs each), default chains per wave.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in msk1 msk2 base msk1 msk2 base; do
  lib=$PWD/build/$v/libffd.so; [ $v = base ] && lib=$PWD/face_alignment_cvpr_2012_amd/lib/libffd.so
  FFD_LIBRARY=$lib timeout -k 10 300 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-host-paths > gpurun_out/msk1_$v.log 2>&1 || { tail -5 gpurun_out/msk1_$v.log; exit 1; }
  echo "$v c4 $(tail -1 gpurun_out/msk1_$v.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(d['value'], 'ms', d['stage_ms_per_step']['meanshift'], 'spot', d['landmark_px_error']['faces_identical'], '/', d['landmark_px_error']['faces_checked'])")"
done
