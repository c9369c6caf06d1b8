#!/bin/bash
# Round 6: rocprofv3 kernel trace of the C3 detector bench (where the detection's 73 ms per 512 frames go).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=$R/gpurun_out/r6/c3prof
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$R/bench.py" --workload c3 --detect --steps 3 --warmup 1 --no-cpu-baseline --no-host-paths > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 "$OUT/trace.log" | cut -c1-300
exit $rc
