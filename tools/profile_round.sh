#!/bin/bash
# Round evidence in one gpurun call: the default bench line (with cpu_baseline), a rocprofv3
# kernel-trace summary of the same command, and two PMC passes (FETCH_SIZE, WRITE_SIZE; separate
# runs, no tracing domains) from which tools/pmc_traffic.py derives per-launch HBM bytes.
# usage: tools/profile_round.sh TAG   -> gpurun_out/round_TAG/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${1:-r1}
OUT=$R/gpurun_out/round_$TAG
mkdir -p "$OUT"
python3 -c "import bench; print(bench.source_digest())" > "$OUT/source_digest.txt"  # the code measured here
BARGS=${BENCH_ARGS:---steps 5 --warmup 2}
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py $BARGS > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.log"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${PROF_TIMEOUT:-420} rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$R/bench.py" $BARGS --no-cpu-baseline > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${PROF_TIMEOUT:-420} rocprofv3 --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/pmc_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
