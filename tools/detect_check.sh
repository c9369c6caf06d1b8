#!/bin/bash
# One gpurun call for the Haar detector: GPU parity tests, the C3 --detect bench line, a rocprofv3
# kernel-trace summary of the same bench.   usage: tools/detect_check.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${1:-det}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_detect.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload c3 --detect --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_bench.log; exit $rc; }
tail -1 gpurun_out/${TAG}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['detect'])"
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o run --output-format csv \
  -- python3 "$R/bench.py" --workload c3 --detect --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/${TAG}_prof.log" 2>&1
echo "rocprof rc=$?"
