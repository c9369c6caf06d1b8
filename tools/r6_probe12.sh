#!/bin/bash
# Round 6: k_meanshift4 register budget (ablib/libffd_ms8.so: <= 64 VGPRs, 8 waves / SIMD; ms7: <= 72) at C4 and C2;
# the detector's compact cascade grid (default build) at C3; the detector GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], 'hp', s['headpose_traverse'], 'ffd', s['ffd_traverse'], 'ms', s['meanshift'], 'err', d.get('landmark_px_error_vs_cpu'), 'det', (d.get('detect') or {}).get('detect_ms_per_step'))" "$1" "$2"; }
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/r6/p12_c4_def_$rep.log 2>&1 || exit $?
  summ gpurun_out/r6/p12_c4_def_$rep.log c4_def
  for tag in ms8 ms7; do
    FFD_LIBRARY=$R/ablib/libffd_$tag.so timeout -k 10 300 python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/r6/p12_c4_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p12_c4_${tag}_$rep.log c4_$tag
  done
  timeout -k 10 300 python3 bench.py --workload c3 --detect --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/r6/p12_c3_$rep.log 2>&1 || exit $?
  summ gpurun_out/r6/p12_c3_$rep.log c3_compact
done
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-paths > gpurun_out/r6/p12_c2.log 2>&1 || exit $?
summ gpurun_out/r6/p12_c2.log c2_def
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_detect.py tests/test_detect.py tests/test_workloads.py > gpurun_out/r6/p12_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6/p12_tests.log; exit $rc
