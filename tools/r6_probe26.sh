#!/bin/bash
# Round 6: traversal block shapes at the round-6 HEAD (env: FFD_TRAV_G_HP / FFD_TRAV_G_FFD; defaults 5x4 / 5x5); C2 x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'hp', s['headpose_traverse'], 'ffd', s['ffd_traverse'], 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  for cfg in def hp4x4 hp3x3 ffd4x4; do
    case $cfg in def) E="";; hp4x4) E="FFD_TRAV_G_HP=4x4";; hp3x3) E="FFD_TRAV_G_HP=3x3";; ffd4x4) E="FFD_TRAV_G_FFD=4x4";; esac
    env $E timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p26_${cfg}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p26_${cfg}_$rep.log "c2 $cfg"
  done
done
