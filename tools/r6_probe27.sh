#!/bin/bash
# Round 6: k_gabor7 with the next input tile loaded into registers during this tile's taps (default) against the
# stage-then-compute form (ablib/libffd_gp0.so); C2 x3 alternating; then the parity / full-batch GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], '7x7', s['gabor_7x7'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2 3; do
  for tag in def gp0; do
    L=""; [ $tag != def ] && L=$R/ablib/libffd_$tag.so
    FFD_LIBRARY=$L timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p27_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p27_${tag}_$rep.log c2_$tag
  done
done
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_full_batch.py tests/test_golden.py > gpurun_out/r6/p27_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6/p27_tests.log; exit $rc
