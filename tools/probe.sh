#!/bin/bash
# Rebuild the library with compile-time probe flags and run the bench once per flag set
# (timing experiments only: probe builds do not produce valid landmarks).
# usage: tools/probe.sh TAG "EXTRA flags 1" "EXTRA flags 2" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out
OUT=gpurun_out/probe_$TAG.jsonl; : > "$OUT"
BARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline}
for extra in "$@"; do
  rm -f face_alignment_cvpr_2012_amd/lib/*.o face_alignment_cvpr_2012_amd/lib/libffd.so
  make -j16 EXTRA="$extra" face_alignment_cvpr_2012_amd/lib/libffd.so > gpurun_out/probe_build.log 2>&1 || { cat gpurun_out/probe_build.log; exit 3; }
  timeout -k 10 ${PASS_TIMEOUT:-200} python bench.py $BARGS > gpurun_out/probe_tmp.log 2>&1
  rc=$?
  cat gpurun_out/probe_tmp.log >> gpurun_out/probe_$TAG.log
  if [ $rc -ne 0 ]; then echo "rc=$rc ($extra)"; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/probe_tmp.log').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(json.dumps({'extra': sys.argv[1], 'value': d['value'], 'ok': d['parity_spot_check'], 'stages': s}))" "$extra" | tee -a "$OUT"
done
