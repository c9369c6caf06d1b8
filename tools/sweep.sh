#!/bin/bash
# Run bench.py once per line of a config file ("ENV=.. ENV2=.." per line); one JSON line each.
# usage: tools/sweep.sh TAG CONFIG_FILE
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; CFG=$2
mkdir -p gpurun_out
OUT=gpurun_out/sweep_$TAG.jsonl; : > "$OUT"
BARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline}
while read -r line; do
  [ -z "$line" ] && continue
  echo "== $line" | tee -a gpurun_out/sweep_$TAG.log
  env $line timeout -k 10 ${PASS_TIMEOUT:-200} python bench.py $BARGS > gpurun_out/sweep_tmp.log 2>&1
  rc=$?
  cat gpurun_out/sweep_tmp.log >> gpurun_out/sweep_$TAG.log
  if [ $rc -ne 0 ]; then echo "rc=$rc" | tee -a gpurun_out/sweep_$TAG.log; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_tmp.log').read().strip().splitlines()[-1]); print(json.dumps({'cfg': sys.argv[1], 'value': d['value'], 'stages': d['stage_ms_per_step'], 'ok': d['parity_spot_check']}))" "$line" | tee -a "$OUT"
done < "$CFG"
