#!/bin/bash
# PMC counter passes over a short bench run (one rocprofv3 process per counter group).
# usage: tools/pmc.sh TAG  (writes gpurun_out/pmc_TAG/<group>/...)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${1:-pmc}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
BARGS=${BENCH_ARGS:---faces 1024 --steps 1 --warmup 1 --no-cpu-baseline --no-host-paths}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 ${PASS_TIMEOUT:-240} rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv \
    -- python3 "$R/bench.py" $BARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc: $grp" | tee -a "$OUT/summary.txt"
  # a counter-name error exits quickly and is harmless; a crash/timeout ends the script
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done < "${PMC_GROUPS:-$R/tools/pmc_groups.txt}"
exit 0
