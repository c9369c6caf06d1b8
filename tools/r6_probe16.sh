#!/bin/bash
# Round 6: the Haar cascade without the stage-0 survivors the invoker's scan skips (default) vs all survivors
# (ablib/libffd_np0.so): C3 detection per 512 frames; then the detector GPU tests on the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], d.get('detect'), 'err', d.get('landmark_px_error_vs_cpu'), d.get('landmark_px_error', {}).get('faces_identical'))" "$1" "$2"; }
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_detect.py tests/test_detect.py > gpurun_out/r6/p16_tests.log 2>&1 || { tail -20 gpurun_out/r6/p16_tests.log; exit 1; }
tail -2 gpurun_out/r6/p16_tests.log
for rep in 1 2; do
  for tag in def np0; do
    L=""; [ $tag != def ] && L=$R/ablib/libffd_$tag.so
    FFD_LIBRARY=$L timeout -k 10 400 python3 bench.py --workload c3 --detect --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/r6/p16_c3_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p16_c3_${tag}_$rep.log c3_$tag
  done
done
