#!/bin/bash
# Round 6: the traversal's rectangle halves in 32-bit registers (default, FFD_RECT_U32=1: no SLP-paired 16-bit ops and
# v_perm_b32 repacks) against the u16 form (ablib/libffd_ru0.so), C2 x3 alternating; C4 x1 each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], d['ms_per_step'], 'hp', s['headpose_traverse'], 'ffd', s['ffd_traverse'], 'ms', s['meanshift'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2 3; do
  for tag in def ru0; do
    L=""; [ $tag != def ] && L=$R/ablib/libffd_$tag.so
    FFD_LIBRARY=$L timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p19_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p19_${tag}_$rep.log c2_$tag
  done
done
for tag in def ru0; do
  L=""; [ $tag != def ] && L=$R/ablib/libffd_$tag.so
  FFD_LIBRARY=$L timeout -k 10 300 python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/r6/p19_c4_${tag}.log 2>&1 || exit $?
  summ gpurun_out/r6/p19_c4_${tag}.log c4_$tag
done
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_full_batch.py > gpurun_out/r6/p19_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r6/p19_tests.log; exit $rc
