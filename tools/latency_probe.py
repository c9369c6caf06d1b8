"""Single-face latency breakdown: analyzeFace (ffd_analyze_faces) wall time and the per-stage
device times of one face, plus small batches.  usage: python tools/latency_probe.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    torch.cuda.init()
    import face_alignment_cvpr_2012_amd as ffd
    from face_alignment_cvpr_2012_amd.synthetic import make_crops
    crops, _ = make_crops(64, seed=9)
    ff = ffd.FaceForest(ffd.FaceForestOptions())
    out = {}
    for n in (1, 4, 16, 64):
        imgs, boxes = list(crops[:n]), [(0, 0, 150, 150)] * n
        ff.analyzeFaces(imgs, boxes)
        ts = []
        for _ in range(20):
            t0 = time.perf_counter()
            ff.analyzeFaces(imgs, boxes)
            ts.append((time.perf_counter() - t0) * 1e3)
        ff.set_profiling(True)
        for _ in range(5):
            ff.analyzeFaces(imgs, boxes)
        st = ff.stage_times()
        ff.set_profiling(False)
        out[n] = {"wall_ms_median": round(float(np.median(ts)), 3),
                  "stages_ms": {k: round(v[0] / 5, 4) for k, v in st.items()},
                  "device_sum_ms": round(sum(v[0] for v in st.values()) / 5, 3)}
    print(json.dumps(out, indent=1))
    ff.close()


if __name__ == "__main__":
    main()
