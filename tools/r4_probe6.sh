#!/bin/bash
# Round 4: walk statistics of the two-walks-per-lane traversal (build/dualst: counts, build/dualph: phases).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name lib extra-args
  FFD_LIBRARY=$PWD/build/$2/libffd.so timeout -k 10 240 python tools/trav_stats.py $3 --out gpurun_out/r4f_$1.json > gpurun_out/r4f_$1.log 2>&1 || { tail -20 gpurun_out/r4f_$1.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r4f_$1.json'))
for k in ('headpose','ffd'): print('$1', k, 'ms=%.2f'%d['stage_ms'][k+'_traverse'][0], {a: (round(b) if b > 10 else round(b, 3)) for a,b in d[k].items()})
"
}
run dualst dualst --dual
run dualph dualph "--dual --phases"
