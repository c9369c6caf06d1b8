"""Time the detector's overflow re-run on crowded frames: 4K and 8K frames tiled with 40-px and
32-px faces (10^4 .. 10^5+ raw detections), one engine.detectFaces call each after a warm-up; the raw
candidate count from engine.detect_candidates.  Prints one JSON line per frame."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import face_alignment_cvpr_2012_amd as ffd  # noqa: E402
import oracle  # noqa: E402
from face_alignment_cvpr_2012_amd.synthetic import load_fixtures  # noqa: E402
from test_gpu_detect import tiled_frame  # noqa: E402

model = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "model", "ffd_model.bin")
fx = load_fixtures()
with ffd.FaceForest(ffd.FaceForestOptions(model_path=model)) as ff:
    for size, h, w in ((40, 2160, 3840), (40, 4320, 7680), (32, 4320, 7680)):
        frame = tiled_frame(fx, oracle, size, h, w)
        n_raw = len(ff.detect_candidates(frame))
        ff.detectFaces([frame])
        t = time.perf_counter()
        boxes = ff.detectFaces([frame])[0]
        ms = (time.perf_counter() - t) * 1e3
        print(json.dumps({"frame": [w, h], "tile": size, "raw_candidates": n_raw, "boxes": len(boxes),
                          "detect_ms": round(ms, 2)}), flush=True)
