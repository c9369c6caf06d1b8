#!/bin/bash
# Round 6: gray / Sobel integrals scanned by the idle eighth wave of the 512-thread Gabor batch workgroups (default)
# against k_integral (ablib/libffd_nofuse.so); C2 bench, then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), {k[6:]: v for k, v in s.items() if k.startswith('gabor')}, 'integral', s['integral_channels'], 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2 3; do
  timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p13_fused_$rep.log 2>&1 || exit $?
  summ gpurun_out/r6/p13_fused_$rep.log fused
  FFD_LIBRARY=$R/ablib/libffd_nofuse.so timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p13_nofuse_$rep.log 2>&1 || exit $?
  summ gpurun_out/r6/p13_nofuse_$rep.log nofuse
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r6/p13_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6/p13_tests.log; exit $rc
