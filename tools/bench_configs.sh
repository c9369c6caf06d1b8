#!/bin/bash
# One bench line per BASELINE.json config at N=1 (C2 default, C3 1080p frames, C4 deep synthetic
# forest, C5 crowd): gpurun_out/configs_TAG/<workload>.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r2}
OUT=gpurun_out/configs_$TAG
mkdir -p "$OUT"
for w in ${WORKLOADS:-c2 c3 c4 c5}; do
  extra=""
  [ "$w" = c3 ] && extra=${C3_ARGS:---detect}  # C3: the GPU Haar detector finds the faces inside the step
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --workload $w $extra ${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu-baseline --no-host-paths} > "$OUT/$w.log" 2>&1
  rc=$?
  echo "$w rc=$rc"
  [ $rc -eq 0 ] || { tail -5 "$OUT/$w.log"; exit $rc; }
  tail -1 "$OUT/$w.log" > "$OUT/$w.json"
done
