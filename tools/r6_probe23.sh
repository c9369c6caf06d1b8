#!/bin/bash
# Round 6: k_integral with the face's gray rows in LDS for batches and the Sobel rows read once per batch (default)
# against the round-6 form (ablib/libffd_ist0.so) and LDS staging alone (ablib/libffd_ist1.so); C2 x2; then the
# whole GPU suite on the default build (9x9 Gabor in the 256-thread 2-column instance too).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'integral', s['integral_channels'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), '9x9', s['gabor_9x9'], 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  for tag in def ist0 ist1; do
    L=""; [ $tag != def ] && L=$R/ablib/libffd_$tag.so
    FFD_LIBRARY=$L timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p23_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p23_${tag}_$rep.log c2_$tag
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r6/p23_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6/p23_tests.log; exit $rc
