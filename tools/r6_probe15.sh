#!/bin/bash
# Round 6: MeanShift's exponential through the 2^(j/32) table (default) vs the 11-step form (ablib/libffd_et0.so),
# C2 and C4; the 2-column 256-thread Gabor instance for 13x13 too (ablib/libffd_s20.so); then the MeanShift /
# workload GPU tests on the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'ms', s.get('meanshift'), 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), {k[6:]: v for k, v in s.items() if k.startswith('gabor')}, 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  for tag in def et0 s20; do
    L=""; [ $tag != def ] && L=$R/ablib/libffd_$tag.so
    FFD_LIBRARY=$L timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p15_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p15_${tag}_$rep.log c2_$tag
  done
  for tag in def et0; do
    L=""; [ $tag != def ] && L=$R/ablib/libffd_$tag.so
    FFD_LIBRARY=$L timeout -k 10 300 python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/r6/p15_c4_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p15_c4_${tag}_$rep.log c4_$tag
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r6/p15_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6/p15_gpu_tests.log
exit $rc
