#!/bin/bash
# Round 6, second lease: (a) bisect the FFD traversal drift -- the C2 bench of round-2..5 commits (abtree/<commit>, each
# worktree with its own build and bench.py) and HEAD on one box; (b) probes: every block staging face 0's planes
# (ablib/libffd_sameplanes.so: the planes always cache-warm), and the pipeline in chunks on 2 streams (the planes of a
# chunk still in the Infinity Cache when its traversals run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], 'hp', s['headpose_traverse'], 'ffd', s['ffd_traverse'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), 'ms', s['meanshift'])" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p2_head_$rep.log 2>&1 || exit $?
  summ gpurun_out/r6/p2_head_$rep.log head
  for wt in r2g 4ac41cc dd0c20d_1 dd0c20d c1b8354 ec50014; do
    (cd abtree/$wt && timeout -k 10 300 python3 bench.py $BA > $R/gpurun_out/r6/p2_${wt}_$rep.log 2>&1) || exit $?
    summ gpurun_out/r6/p2_${wt}_$rep.log $wt
  done
  FFD_LIBRARY=$R/ablib/libffd_sameplanes.so timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p2_sameplanes_$rep.log 2>&1 || exit $?
  summ gpurun_out/r6/p2_sameplanes_$rep.log sameplanes
done
for cfg in "2 256" "2 512" "3 128" "2 1024"; do
  set -- $cfg
  FFD_STREAMS=$1 FFD_CHUNK=$2 timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p2_s$1_c$2.log 2>&1 || exit $?
  summ gpurun_out/r6/p2_s$1_c$2.log "streams$1_chunk$2"
done
echo done
