#!/bin/bash
# Round 6: the 2-column Gabor instance in 256-thread workgroups (4-row bands): ablib/libffd_s25.so (25x25),
# s1319 (13x13 + 19x19 instead of the 512-thread form), s28 (all three) against the default; C2 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), {k[6:]: v for k, v in s.items() if k.startswith('gabor')}, 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p14_def_$rep.log 2>&1 || exit $?
  summ gpurun_out/r6/p14_def_$rep.log def
  for tag in s25 s1319 s28; do
    FFD_LIBRARY=$R/ablib/libffd_$tag.so timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p14_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p14_${tag}_$rep.log $tag
  done
done
echo done
