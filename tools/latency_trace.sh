#!/bin/bash
# Single-face latency timeline: examples/build/bench_host on one 150x150 crop (the reference's
# one-analyzeFace-per-call pattern, eval_ffd.cpp:89) under rocprofv3 kernel + memory-copy traces.
# usage: tools/latency_trace.sh TAG   -> gpurun_out/lat_TAG/{run_kernel_trace.csv, ...}
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=${1:-a}
OUT=$R/gpurun_out/lat_$TAG
mkdir -p "$OUT"
python3 -c "
from face_alignment_cvpr_2012_amd.synthetic import make_crops
c, _ = make_crops(4, seed=9); c.tofile('$OUT/crops.bgr')"
timeout -k 10 60 "$R/examples/build/bench_host" "$R/model/ffd_model.bin" "$OUT/crops.bgr" 1 150 150 20 > "$OUT/plain.json" 2>&1
rc=$?; echo "plain rc=$rc"; cat "$OUT/plain.json"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/trace" -o run --output-format csv \
  -- "$R/examples/build/bench_host" "$R/model/ffd_model.bin" "$OUT/crops.bgr" 1 150 150 5 > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
rm -f "$OUT/crops.bgr"
