#!/bin/bash
# Round 4: k_meanshift4 votes per lane per tile (FFD_MS_K 2 / 4 / 8) at C4 and C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in base msk2 msk8; do
  lib=$PWD/build/$v/libffd.so; [ $v = base ] && lib=$PWD/face_alignment_cvpr_2012_amd/lib/libffd.so
  for w in c4 c2; do
    FFD_LIBRARY=$lib timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-host-paths > gpurun_out/msk_$v$w.log 2>&1 || { tail -5 gpurun_out/msk_$v$w.log; exit 1; }
    echo "$v $w $(tail -1 gpurun_out/msk_$v$w.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(d['value'], 'ms', d['stage_ms_per_step']['meanshift'], 'spot', d['landmark_px_error']['faces_identical'], '/', d['landmark_px_error']['faces_checked'])")"
  done
done
