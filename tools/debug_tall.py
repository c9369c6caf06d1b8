"""Debug: the per-stage trace of a very tall face (GPU vs oracle), first mismatching stage."""
import sys
import numpy as np
sys.path.insert(0, ".")
import face_alignment_cvpr_2012_amd as ffd
import oracle
from face_alignment_cvpr_2012_amd.synthetic import load_fixtures
import torch
torch.cuda.init()
fx = load_fixtures()
img = fx["images"][0]
box = tuple(int(v) for v in sys.argv[1:5]) if len(sys.argv) > 4 else (100, 5, 20, 240)
oracle.load_model("model/ffd_model.bin")
with ffd.FaceForest(ffd.FaceForestOptions(model_path="model/ffd_model.bin")) as ff:
    f = ff.analyzeFaces([img], [box], [0])[0]
    g = ff.trace(0, box[2], box[3])
r, o = oracle.analyze_face(img, box, threads=8, trace=True)
print("headpose", f.headpose, r["headpose"], "var", f.pose_variance, r["pose_variance"])
for k in ("face", "channels", "hp_leaves", "pose_freq", "trees", "vote_counts", "ms_mean"):
    a, b = g[k], o[k]
    same = a.shape == b.shape and np.array_equal(a, b)
    print(k, a.shape, b.shape, "same" if same else "DIFF")
    if not same and a.shape == b.shape:
        d = np.argwhere(a != b)
        print("  n diff", len(d), "first", d[:5].tolist(), "last", d[-3:].tolist())
        if k == "channels":
            for c in sorted(set(d[:, 0].tolist()))[:10]:
                dc = d[d[:, 0] == c]
                print("   ch", c, "rows", dc[:, 1].min(), dc[:, 1].max(), "cols", dc[:, 2].min(), dc[:, 2].max(), "n", len(dc))
