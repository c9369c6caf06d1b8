#!/bin/bash
# Kernel + HIP API trace of examples/evaluate_mt on C2 face 0 (the reference's per-patch evaluateMT pattern):
# where a sample's first evaluateMT call (the grid evaluation) spends its time.  -> gpurun_out/emt/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out/emt
python3 - <<'PY' > gpurun_out/emt/args.txt
import sys; sys.path.insert(0, ".")
import numpy as np, bench
wl = bench.make_workload("c2", 0, 1, 1, 1)
img, box = wl.face(0)
np.ascontiguousarray(img).tofile("gpurun_out/emt/face0.bgr")
print(img.shape[1], img.shape[0], *[int(v) for v in box])
PY
cd /tmp && export TMPDIR=/tmp
FFD_EVAL_REPS=3 timeout -k 10 120 rocprofv3 --kernel-trace --hip-trace --stats -d "$R/gpurun_out/emt/trace" -o run \
  --output-format csv -- "$R/examples/build/evaluate_mt" "$R/model/ffd_model.bin" --crop "$R/gpurun_out/emt/face0.bgr" \
  $(cat "$R/gpurun_out/emt/args.txt") > "$R/gpurun_out/emt/out.log" 2>&1
rc=$?; tail -2 "$R/gpurun_out/emt/out.log"; rm -f "$R/gpurun_out/emt/face0.bgr"; exit $rc
