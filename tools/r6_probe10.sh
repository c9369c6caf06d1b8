#!/bin/bash
# Round 6: head-pose faces in interleaved pairs with plane touches (default) against interleaved without touches
# (ablib/libffd_hpnt.so) and face-major without touches (ablib/libffd_hpi1.so, the previous form); C2 bench, then C4
# and C3 (detector) lines and the whole GPU suite on the default build (Gabor 13x13 / 19x19 with 2-column threads).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], 'hp', s['headpose_traverse'], 'ffd', s['ffd_traverse'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), {k[6:]: v for k, v in s.items() if k.startswith('gabor')}, 'ms', s['meanshift'], 'err', d.get('landmark_px_error_vs_cpu'), 'det', (d.get('detect') or {}).get('detect_ms_per_step'))" "$1" "$2"; }
BA="--steps 10 --warmup 3 --no-cpu-baseline --no-host-paths"
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p10_def_$rep.log 2>&1 || exit $?
  summ gpurun_out/r6/p10_def_$rep.log hpilv2_touch
  for tag in hpnt hpi1; do
    FFD_LIBRARY=$R/ablib/libffd_$tag.so timeout -k 10 300 python3 bench.py $BA > gpurun_out/r6/p10_${tag}_$rep.log 2>&1 || exit $?
    summ gpurun_out/r6/p10_${tag}_$rep.log $tag
  done
done
timeout -k 10 300 python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/r6/p10_c4.log 2>&1 || exit $?
summ gpurun_out/r6/p10_c4.log c4
timeout -k 10 300 python3 bench.py --workload c3 --detect --steps 5 --warmup 2 --no-cpu-baseline --no-host-paths > gpurun_out/r6/p10_c3.log 2>&1 || exit $?
summ gpurun_out/r6/p10_c3.log c3
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r6/p10_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6/p10_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/r6_probe11.sh
