#!/bin/bash
# Round 6: chunked C2 batches (FFD_CHUNK faces per chunk, FFD_STREAMS workspaces) — planes of a chunk of 128-256 faces
# fit the 256 MB Infinity Cache between the channel kernels and the traversals.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'hp', s['headpose_traverse'], 'ffd', s['ffd_traverse'], 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  for cfg in "def" "512 1" "256 1" "512 2" "256 2" "1024 2"; do
    set -- $cfg
    if [ "$1" = def ]; then E=""; else E="FFD_CHUNK=$1 FFD_STREAMS=$2"; fi
    env $E timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p20_${1}_${2:-x}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p20_${1}_${2:-x}_$rep.log "c2 chunk=$cfg"
  done
done
