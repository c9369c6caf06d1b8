#!/bin/bash
# Round 6: k_meanshift4 software-pipelined tiles (default FFD_MS4_PIPE=1: sums of tile i beside the terms of tile
# i + 1, branch-free) vs the phased form (ablib/libffd_p0.so) and the pipelined form at one vote per lane per tile
# (ablib/libffd_pk1.so); C4 x2 alternating, then the MeanShift / workload GPU tests on the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'ms', s['meanshift'], 'err', d.get('landmark_px_error_vs_cpu'), d.get('landmark_px_error', {}).get('faces_identical'))" "$1" "$2"; }
for rep in 1 2; do
  for tag in def p0 pk1; do
    L=""; [ $tag != def ] && L=$R/ablib/libffd_$tag.so
    FFD_LIBRARY=$L timeout -k 10 300 python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/r6/p21_c4_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p21_c4_${tag}_$rep.log c4_$tag
  done
done
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_workloads.py tests/test_full_batch.py tests/test_options.py tests/test_gpu_parity.py > gpurun_out/r6/p21_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6/p21_tests.log; exit $rc
