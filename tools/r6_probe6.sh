#!/bin/bash
# Round 6: traversal plane touches FFD_TRAV_TOUCH 2 (default) against 0 (off), 1, 3 and the same-planes probe, C2 bench;
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], 'hp', s['headpose_traverse'], 'ffd', s['ffd_traverse'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), 'ms', s['meanshift'], 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p6_pfw_$rep.log 2>&1 || exit $?
  summ gpurun_out/r6/p6_pfw_$rep.log touch2
  for tag in touch0 touch1 touch3 sameplanes; do
    FFD_LIBRARY=$R/ablib/libffd_$tag.so timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p6_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p6_${tag}_$rep.log $tag
  done
done
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_full_batch.py tests/test_golden.py tests/test_gpu_parity.py tests/test_workloads.py tests/test_api_edges.py tests/test_fint_window.py tests/test_engine_choice.py > gpurun_out/r6/p6_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6/p6_tests.log; exit $rc
