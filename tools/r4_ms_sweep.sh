#!/bin/bash
# Round 4: k_meanshift4's chains per wave at C4 (FFD_MS_WAVES: the fewest waves the choice must give), default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wv in 4096 2048 1024 8192; do
  FFD_MS_WAVES=$wv timeout -k 10 300 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-host-paths > gpurun_out/ms_w$wv.log 2>&1 || { tail -5 gpurun_out/ms_w$wv.log; exit 1; }
  echo "ms_waves=$wv $(tail -1 gpurun_out/ms_w$wv.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(d['value'], 'ms', d['stage_ms_per_step']['meanshift'], 'spot', d['landmark_px_error']['faces_identical'], '/', d['landmark_px_error']['faces_checked'])")"
done
