#!/bin/bash
# Round 6: the separable Gabor scales with 2 output columns per H-pass thread (512-thread workgroups, <= 128 VGPRs:
# ablib/libffd_g{19,13,1319,25,25w3}.so = which scales) against the 4-column default, C2 bench (per-scale stage
# times, landmark parity vs the goldens); C4 with the touch gating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], 'ffd', s['ffd_traverse'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), {k[6:]: v for k, v in s.items() if k.startswith('gabor')}, 'ms', s['meanshift'], 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p9_def_$rep.log 2>&1 || exit $?
  summ gpurun_out/r6/p9_def_$rep.log cpt4
  for tag in g19 g13 g1319 g25 g25w3; do
    FFD_LIBRARY=$R/ablib/libffd_$tag.so timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p9_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p9_${tag}_$rep.log $tag
  done
done
timeout -k 10 300 python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/r6/p9_c4.log 2>&1 || exit $?
summ gpurun_out/r6/p9_c4.log c4
echo done
