#!/bin/bash
# k_haar_cascade time (rocprofv3 kernel trace of the C3 --detect bench) for the default build and for
# each probe_libs/libffd_TAG.so; probe builds may break the detections, so the bench's exit status is
# not checked, only the trace.  usage: tools/casc_probe.sh TAG [TAG ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
for tag in base "$@"; do
  lib=$R/probe_libs/libffd_$tag.so
  [ "$tag" = base ] && lib=$R/face_alignment_cvpr_2012_amd/lib/libffd.so
  (cd /tmp && export TMPDIR=/tmp && FFD_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/cp_$tag" -o run \
    --output-format csv -- python3 "$R/bench.py" --workload c3 --detect --steps 1 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/cp_$tag.log" 2>&1)
  rc=$?; [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
  python3 - "$R/gpurun_out/cp_$tag/run_kernel_stats.csv" "$tag" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'haar_cascade' in r['Name']:
        print(sys.argv[2], 'k_haar_cascade avg ms', round(float(r['AverageNs']) / 1e6, 3), 'calls', r['Calls'])
PY
done
