#!/bin/bash
# Run the bench once per prebuilt probe_libs/libffd_TAG.so (FFD_LIBRARY), one JSON summary line each.
#   tools/run_variants.sh OUT TAG [TAG ...]   (BENCH_ARGS overrides the bench flags)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift
mkdir -p gpurun_out; : > "$OUT.jsonl"
BARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-host-paths}
for tag in "$@"; do
  lib=$PWD/probe_libs/libffd_$tag.so
  [ "$tag" = base ] && lib=$PWD/face_alignment_cvpr_2012_amd/lib/libffd.so
  FFD_LIBRARY=$lib timeout -k 10 ${PASS_TIMEOUT:-200} python bench.py $BARGS > gpurun_out/variant_tmp.log 2>&1
  rc=$?
  cat gpurun_out/variant_tmp.log >> "$OUT.log"
  if [ $rc -ne 0 ]; then echo "rc=$rc ($tag)"; tail -5 gpurun_out/variant_tmp.log; exit $rc; fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/variant_tmp.log').read().strip().splitlines()[-1]); print(json.dumps({'tag': sys.argv[1], 'value': d['value'], 'same': d.get('landmark_px_error',{}).get('faces_identical'), 'stages': d['stage_ms_per_step']}))" "$tag" | tee -a "$OUT.jsonl"
done
