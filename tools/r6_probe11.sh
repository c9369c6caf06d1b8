#!/bin/bash
# Round 6: detector frames per group (FFD_DETECT_GROUP: the pyramid / integral / cascade working set of a group; 64
# frames of 1080p ~2.6 GB, 4 ~160 MB, inside the Infinity Cache), C3 --detect bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], 'det', (d.get('detect') or {}).get('detect_ms_per_step'), 'faces', (d.get('detect') or {}).get('faces_found'))" "$1" "$2"; }
for g in 64 32 16 8 4 64; do
  FFD_DETECT_GROUP=$g timeout -k 10 300 python3 bench.py --workload c3 --detect --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/r6/p11_g$g.log 2>&1 || exit $?
  summ gpurun_out/r6/p11_g$g.log group$g
done
