#!/bin/bash
# Round 4: per-step timing of the deep walk (test vs record wait), FFD_TRAV_STATS=2 builds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in t2 t2p6 t2p2; do
  FFD_LIBRARY=$PWD/build/$v/libffd.so timeout -k 10 240 python tools/trav_stats.py --timing --out gpurun_out/trav_timing_$v.json > gpurun_out/trav_timing_$v.log 2>&1 || { tail -20 gpurun_out/trav_timing_$v.log; exit 1; }
  echo "== $v"; python3 -c "
import json; d=json.load(open('gpurun_out/trav_timing_$v.json'))
for k in ('headpose','ffd'): print(k, 'ms=%.2f'%d['stage_ms'][k+'_traverse'][0], {a: round(b) for a,b in d[k].items()})
"
done
