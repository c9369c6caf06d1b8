"""Generate tests/golden/oracle_golden.npz: expected outputs of the CPU restatement (oracle/)
on the 20 bundled faces and 8 seeded C2 crops (golden vectors generated
here by the build's own restatement).  Committed, so the GPU box checks the engine against
fixed vectors without re-running the oracle, and the CPU suite pins the oracle against drift.

Per case: headpose, pose variance, n_trees, 10 landmarks, selected tree ids, MeanShift means,
vote counts, and CRC32 digests of the scaled face, the 38 integral channels and the HP / FFD
leaf arrays (reference order, [patch][tree]).

usage: python tests/golden/make_oracle_golden.py   (needs model/ffd_model.bin + oracle build)
"""
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

N_CROPS = 8
CROP_SEED = 77


def cases():
    d = np.load(os.path.join(HERE, "faces.npz"))
    out = [(d["images"][i], tuple(int(v) for v in d["boxes"][i])) for i in range(len(d["images"]))]
    from face_alignment_cvpr_2012_amd.synthetic import make_crops
    crops, _ = make_crops(N_CROPS, seed=CROP_SEED)
    out += [(c, (0, 0, c.shape[1], c.shape[0])) for c in crops]
    return out


def crc(a):
    return np.uint32(zlib.crc32(np.ascontiguousarray(a).tobytes()) & 0xFFFFFFFF)


def record(face, tr):
    return dict(headpose=np.float32(face["headpose"]), pose_variance=np.float32(face["pose_variance"]),
                n_trees=np.int32(face["n_trees"]), points=face["points"].astype(np.int32),
                trees=np.pad(tr["trees"], (0, 32 - len(tr["trees"])), constant_values=-1).astype(np.int32),
                ms_mean=tr["ms_mean"].astype(np.float32), vote_counts=tr["vote_counts"].astype(np.int32),
                crc_face=crc(tr["face"]), crc_channels=crc(tr["channels"].astype(np.uint32)),
                crc_hp_leaves=crc(tr["hp_leaves"].astype(np.int32)),
                crc_mp_leaves=crc(tr["mp_leaves"].astype(np.int32)))


def main():
    import oracle
    oracle.load_model(os.path.join(REPO, "model", "ffd_model.bin"))
    recs = []
    for img, box in cases():
        face, tr = oracle.analyze_face(img, box, threads=8, trace=True)
        recs.append(record(face, tr))
    out = {k: np.stack([r[k] for r in recs]) for k in recs[0]}
    out["n_fixtures"] = np.int32(20)
    out["crop_seed"] = np.int32(CROP_SEED)
    np.savez_compressed(os.path.join(HERE, "oracle_golden.npz"), **out)
    print("wrote", len(recs), "cases")


if __name__ == "__main__":
    main()
