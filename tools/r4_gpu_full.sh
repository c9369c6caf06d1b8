#!/bin/bash
# Round 4: the whole GPU suite, smoke(), then the default bench (C2) with its host paths.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r4}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/tests_$TAG.log 2>&1
rc=$?; grep -E 'passed|failed|error' gpurun_out/tests_$TAG.log | tail -3; [ $rc -eq 0 ] || { grep -E 'FAILED|Error|assert' gpurun_out/tests_$TAG.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { tail -5 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms_per_step']
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'hp', s['headpose_traverse'], 'ffd', s['ffd_traverse'], 'ms', s['meanshift'], 'spot', d['landmark_px_error'].get('faces_identical'), 'host_incl', d.get('host_inclusive',{}).get('value'))
print('evaluate_mt', d.get('evaluate_mt_path'))"
