#!/bin/bash
# Round 4: row-run staging (build/rows) and pair walkers (build/pair) against the in-tree build: leaves on every
# C2 face and 512 C4 faces, stage times, walk phases.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VARIANTS="${VARIANTS:-rows pair}" tools/r4_probe5.sh || exit 1
for v in ${PHASES-rowsph pairph}; do
  FFD_LIBRARY=$PWD/build/$v/libffd.so timeout -k 10 240 python tools/trav_stats.py --phases --out gpurun_out/r4g_$v.json > gpurun_out/r4g_$v.log 2>&1 || { tail -20 gpurun_out/r4g_$v.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r4g_$v.json'))
for k in ('headpose','ffd'): print('$v', k, 'ms=%.2f'%d['stage_ms'][k+'_traverse'][0], {a: round(b) for a,b in d[k].items()})
"
done
