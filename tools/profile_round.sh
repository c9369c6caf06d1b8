#!/bin/bash
# Round evidence in one gpurun call (C2, the bench's default workload):
#   1. a rocprofv3 kernel-trace summary of the bench (kernel_stats.csv);
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, no tracing domains) -> traffic.json
#      via tools/pmc_traffic.py, stamped with the source digest of the code measured;
#   3. the bench line itself (with cpu_baseline and the host paths), which quotes `traffic` from
#      that traffic.json (copied into profiles/TAG/ on the box, where bench.py looks for it).
# The profiled runs skip the host-inclusive / latency measurements so every launch is a full batch.
# usage: tools/profile_round.sh TAG   -> gpurun_out/round_TAG/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${1:-r1}
OUT=$R/gpurun_out/round_$TAG
mkdir -p "$OUT"
python3 -c "import bench; print(bench.source_digest())" > "$OUT/source_digest.txt"  # the code measured here
BARGS=${BENCH_ARGS:---steps 5 --warmup 2}
PARGS="--no-cpu-baseline --no-host-paths"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${PROF_TIMEOUT:-420} rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$R/bench.py" $BARGS $PARGS > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${PROF_TIMEOUT:-420} rocprofv3 --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 1 --warmup 1 $PARGS > "$OUT/pmc_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cd "$R"
python3 tools/pmc_traffic.py "$OUT" "$OUT/traffic.json" c2 4096 > /dev/null || exit 5
mkdir -p "profiles/$TAG" && cp "$OUT/traffic.json" "profiles/$TAG/traffic.json"
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py $BARGS > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.log"
exit $rc
