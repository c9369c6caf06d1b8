#!/bin/bash
# Round 6: traversal touch variants (default distance 1; 64-B sectors; no head-pose touches; touches before the
# staging loads; off) on the C2 bench, one full bench line (host paths: evaluate_mt pattern with tree-grouped
# single-face grids), then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; e=d.get('evaluate_mt_path') or {}; print(sys.argv[2], d['value'], 'hp', s['headpose_traverse'], 'ffd', s['ffd_traverse'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), 'ms', s['meanshift'], 'err', d.get('landmark_px_error_vs_cpu'), 'emt', e.get('first_call_ms'), e.get('all_calls_ms'), e.get('calls_vs_batched_per_face'), 'lat', (d.get('analyze_face_latency') or {}).get('median_ms'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p8_def_$rep.log 2>&1 || exit $?
  summ gpurun_out/r6/p8_def_$rep.log touch1
  for tag in sect2 nohp first touch0; do
    FFD_LIBRARY=$R/ablib/libffd_$tag.so timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p8_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p8_${tag}_$rep.log $tag
  done
done
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6/p8_full.log 2>&1 || exit $?
summ gpurun_out/r6/p8_full.log full
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r6/p8_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6/p8_tests.log; exit $rc
