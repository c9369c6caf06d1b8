#!/bin/bash
# Round-6 HEAD snapshot in one lease: two quick C2 benches, the whole GPU suite, tools/profile_round.sh (rocprofv3
# kernel trace, FETCH_SIZE / WRITE_SIZE passes, the full bench line) and tools/bench_configs.sh (C2..C5).
# usage: tools/r6_snapshot.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r6b}
mkdir -p gpurun_out/r6
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(sys.argv[2], d['value'], 'hp', s['headpose_traverse'], 'ffd', s['ffd_traverse'], 'gabor', round(sum(v for k,v in s.items() if k.startswith('gabor')),3), 'ms', s['meanshift'], 'err', d.get('landmark_px_error_vs_cpu'))" "$1" "$2"; }
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-paths > gpurun_out/r6/snap_$rep.log 2>&1 || exit $?
  summ gpurun_out/r6/snap_$rep.log quick
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r6/snap_tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/r6/snap_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh $TAG || exit $?
bash tools/bench_configs.sh $TAG || exit $?
echo done
