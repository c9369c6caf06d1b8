#!/bin/bash
# Round 4: MeanShift form at C2 re-measured after the k_meanshift4 K=2 change (env overrides only, HEAD library):
# default (k_meanshift, path 1) vs k_meanshift4 at 4,096 / 8,192 / 2,048 waves.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload c2 --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/msc2_$tag.log 2>&1 || { tail -5 gpurun_out/msc2_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/msc2_$tag.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(d['value'], 'ms', d['stage_ms_per_step']['meanshift'], 'spot', d['landmark_px_error']['faces_identical'], '/', d['landmark_px_error']['faces_checked'])")"
}
if [ "${1:-}" = c2 ]; then  # chains per wave 2 (20,480 waves) at C2
  run base FFD_MS_KERNEL=0
  run ms4c2 FFD_MS_KERNEL=4 FFD_MS_WAVES=16384
  run base2 FFD_MS_KERNEL=0
  run ms4c2b FFD_MS_KERNEL=4 FFD_MS_WAVES=16384
  exit 0
fi
run base FFD_MS_KERNEL=0
run ms4 FFD_MS_KERNEL=4
run ms4w8k FFD_MS_KERNEL=4 FFD_MS_WAVES=8192
run ms4w2k FFD_MS_KERNEL=4 FFD_MS_WAVES=2048
run base2 FFD_MS_KERNEL=0
