#!/bin/bash
# Round 6: k_gray_resize with the face's source box converted to gray into LDS first and a thread per output column
# (default) against the per-pixel form (ablib/libffd_grs0.so, FFD_GRAY_STAGE_MAX=0); C2 x3 alternating, C3 x1;
# then the parity / full-batch / workload GPU tests on the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'gray', s['gray_resize'], 'integral', s['integral_channels'], 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  for tag in def grs0; do
    L=""; [ $tag != def ] && L=$R/ablib/libffd_$tag.so
    FFD_LIBRARY=$L timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p24_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p24_${tag}_$rep.log c2_$tag
  done
done
for tag in def grs0; do
  L=""; [ $tag != def ] && L=$R/ablib/libffd_$tag.so
  FFD_LIBRARY=$L timeout -k 10 400 python3 bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/r6/p24_c3_${tag}.log 2>&1 || exit $?
  summ gpurun_out/r6/p24_c3_${tag}.log c3_$tag
done
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_full_batch.py tests/test_workloads.py tests/test_golden.py tests/test_api_edges.py > gpurun_out/r6/p24_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6/p24_tests.log; exit $rc
