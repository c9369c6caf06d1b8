"""MeanShift stage time vs iteration cap (timing probe; results are not the reference's when capped)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import face_alignment_cvpr_2012_amd as ffd  # noqa: E402
from face_alignment_cvpr_2012_amd.synthetic import make_crops  # noqa: E402

crops, _ = make_crops(4096, seed=2012)
d = torch.from_numpy(np.ascontiguousarray(crops)).cuda()
out = torch.zeros(4096 * 112, dtype=torch.uint8, device="cuda")
boxes = np.tile(np.array([[0, 0, 150, 150]], np.int32), (4096, 1))
for it in (0, 1, 2, 4, 7):
    ff = ffd.FaceForest(ffd.FaceForestOptions(ms_option=ffd.MeanShiftOption(max_iterations=it)))
    for _ in range(2):
        ff.analyze_device(d.data_ptr(), 150 * 150 * 3, 150, 150, 450, 4096, boxes, np.arange(4096, dtype=np.int32),
                          out.data_ptr())
    ff.synchronize()
    ff.set_profiling(True)
    for _ in range(3):
        ff.analyze_device(d.data_ptr(), 150 * 150 * 3, 150, 150, 450, 4096, boxes, np.arange(4096, dtype=np.int32),
                          out.data_ptr())
    ff.synchronize()
    st = ff.stage_times()
    print("max_iterations", it, "meanshift ms", round(st["meanshift"][0] / 3, 3), "votes ms", round(st["votes"][0] / 3, 3),
          flush=True)
    ff.close()
