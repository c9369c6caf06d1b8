#!/bin/bash
# Round 4: engine environment knobs on the default build (no rebuild): channel streams (the Gabor scales and the
# integrals side by side on fork streams within a chunk).  One bench line per setting.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cs in 1 2 3 6; do
  FFD_CHANNEL_STREAMS=$cs timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/env_cs$cs.log 2>&1 || { tail -5 gpurun_out/env_cs$cs.log; exit 1; }
  echo "channel_streams=$cs $(tail -1 gpurun_out/env_cs$cs.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
s = d['stage_ms_per_step']
print(d['value'], d['ms_per_step'], 'spot', d['landmark_px_error']['faces_identical'], {k: s[k] for k in ('gabor_25x25','gabor_7x7','integral_channels','headpose_traverse')})")"
done
