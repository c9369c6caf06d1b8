#!/bin/bash
# Like tools/probe.sh, but each argument is "EXTRA compile flags::ENV=a ENV2=b" (either part may be
# empty): rebuild libffd.so with the flags, run the bench under the env, one JSON line per config.
# usage: tools/probe2.sh TAG "flags::env" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out
OUT=gpurun_out/probe2_$TAG.jsonl; : > "$OUT"
BARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-host-paths}
last="__none__"
for cfg in "$@"; do
  extra=${cfg%%::*}; envs=${cfg#*::}
  if [ "$extra" != "$last" ]; then
    rm -f face_alignment_cvpr_2012_amd/lib/ffd_kernels.o face_alignment_cvpr_2012_amd/lib/libffd.so
    make -j16 EXTRA="$extra" face_alignment_cvpr_2012_amd/lib/libffd.so > gpurun_out/probe2_build.log 2>&1 || { tail -20 gpurun_out/probe2_build.log; exit 3; }
    last=$extra
  fi
  env $envs timeout -k 10 ${PASS_TIMEOUT:-200} python bench.py $BARGS > gpurun_out/probe2_tmp.log 2>&1
  rc=$?
  cat gpurun_out/probe2_tmp.log >> gpurun_out/probe2_$TAG.log
  if [ $rc -ne 0 ]; then echo "rc=$rc ($cfg)"; tail -5 gpurun_out/probe2_tmp.log; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/probe2_tmp.log').read().strip().splitlines()[-1]); s=d['stage_ms_per_step']; print(json.dumps({'cfg': sys.argv[1], 'value': d['value'], 'ok': d.get('landmark_px_error',{}).get('faces_identical'), 'hp': s['headpose_traverse'], 'ffd': s['ffd_traverse'], 'ms': d['ms_per_step']}))" "$cfg" | tee -a "$OUT"
done
