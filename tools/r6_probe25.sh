#!/bin/bash
# Round 6: the vote filter's pipeline depth (FFD_VOTE_U batches of 64 items per group: 2 default, 3 / 4 in
# ablib/libffd_vu3.so / libffd_vu4.so); C2 x2 alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'votes', s['votes'], 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  for tag in def vu3 vu4; do
    L=""; [ $tag != def ] && L=$R/ablib/libffd_$tag.so
    FFD_LIBRARY=$L timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p25_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p25_${tag}_$rep.log c2_$tag
  done
done
