"""Generate tests/golden/c2_golden.npz: the CPU restatement's (oracle/) result for EVERY face of
the bench's C2 batch (BASELINE.json configs[1]: 4,096 synthetic 150x150 crops, seed 2012 = rank 0
of bench.py), so the GPU suite and bench.py compare the whole batch, not a sample.

Per face: headpose and pose variance (float32 bits), n_trees, 10 landmarks (int16, bbox-relative
= crop coordinates).  Also the CRC32 of the generated crops, so a test can tell a drifted crop
generator from an engine mismatch, and the crops' ground-truth landmarks (synthetic.crop_ground_truth)
for the px error against the annotations.

usage: python tests/golden/make_c2_golden.py   (needs model/ffd_model.bin + the oracle build; about
a minute on 8 host threads)
"""
import concurrent.futures as cf
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

N_FACES = 4096
SEED = 2012
CROP = 150


def main():
    import oracle
    from face_alignment_cvpr_2012_amd.synthetic import crop_ground_truth, make_crops
    oracle.load_model(os.path.join(REPO, "model", "ffd_model.bin"))
    crops, _ = make_crops(N_FACES, seed=SEED)
    box = (0, 0, CROP, CROP)
    with cf.ThreadPoolExecutor(os.cpu_count() or 8) as ex:  # ctypes drops the GIL: one face per thread
        faces = list(ex.map(lambda c: oracle.analyze_face(c, box, threads=1)[0], crops))
    out = dict(
        headpose=np.array([f["headpose"] for f in faces], np.float32),
        pose_variance=np.array([f["pose_variance"] for f in faces], np.float32),
        n_trees=np.array([f["n_trees"] for f in faces], np.int8),
        points=np.stack([f["points"] for f in faces]).astype(np.int16),
        ground_truth=crop_ground_truth(N_FACES, seed=SEED).astype(np.float32),
        crops_crc=np.uint32(zlib.crc32(crops.tobytes()) & 0xFFFFFFFF),
        seed=np.int32(SEED),
    )
    np.savez_compressed(os.path.join(HERE, "c2_golden.npz"), **out)
    print("wrote", N_FACES, "faces; crops crc", hex(int(out["crops_crc"])))


if __name__ == "__main__":
    main()
