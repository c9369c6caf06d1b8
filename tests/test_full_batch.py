"""Every face of each config's bench batch against the CPU restatement.

C2 (BASELINE.json configs[1]): all 4,096 crops of bench.py's rank-0 batch (seed 2012) against the
committed oracle goldens (tests/golden/c2_golden.npz, tests/golden/make_c2_golden.py), through both
host entry points: ffd_analyze_faces (host images, the C++ shim's call) and ffd_analyze_faces_device
(images resident in HBM, the bench's call).  Bar: landmarks, n_trees and the headpose / pose-variance
float bits identical for every face (eval_ffd.cpp:102-108's inputs).
C3: the bench's first 1080p frame (seed 1080) with all 8 detectFace-enlarged boxes.
C5: the bench's first 64-face frame (crops seed 5000), and 64 boxes on one image, every face.
"""
import os
import zlib

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "c2_golden.npz")
CROP = 150


@pytest.fixture(scope="module")
def c2():
    from face_alignment_cvpr_2012_amd.synthetic import make_crops
    g = np.load(GOLDEN, allow_pickle=False)
    crops, _ = make_crops(int(g["points"].shape[0]), seed=int(g["seed"]))
    return crops, {k: g[k] for k in g.files}


def test_c2_golden_matches_generator(c2):
    """The committed goldens describe exactly the crops the generator makes (a drifted generator
    fails here, not as an engine mismatch), and the ground truth is the annotated landmarks."""
    from face_alignment_cvpr_2012_amd.synthetic import crop_ground_truth
    crops, g = c2
    assert crops.shape == (4096, CROP, CROP, 3)
    assert zlib.crc32(crops.tobytes()) & 0xFFFFFFFF == int(g["crops_crc"])
    np.testing.assert_allclose(g["ground_truth"], crop_ground_truth(4096, seed=int(g["seed"])), atol=1e-4)
    assert (g["n_trees"] == 20).all()


def test_c2_golden_matches_oracle_sample(c2, oracle_mod):
    """The oracle reproduces its committed goldens (16 faces spread over the batch)."""
    crops, g = c2
    for k in np.linspace(0, 4095, 16).astype(int):
        ref, _ = oracle_mod.analyze_face(crops[k], (0, 0, CROP, CROP), threads=8)
        np.testing.assert_array_equal(ref["points"], g["points"][k], err_msg=f"face {k}")
        assert np.float32(ref["headpose"]).tobytes() == g["headpose"][k].tobytes(), k


def test_c2_golden_px_error_band(c2):
    """The restatement's mean landmark error against the crops' annotations (the metric's
    'mean landmark px error' versus ground truth) sits in the band of the 20 fixtures' IOD error."""
    _, g = c2
    err = np.linalg.norm(g["points"].astype(np.float64) - g["ground_truth"], axis=2)
    assert 2.5 < err.mean() < 5.0


def _compare(faces_pts, hp, var, nt, g, label):
    bad = np.nonzero((faces_pts != g["points"]).any(axis=(1, 2)))[0]
    assert bad.size == 0, f"{label}: {bad.size} faces differ, first {bad[:8].tolist()}"
    np.testing.assert_array_equal(hp.view(np.uint32), g["headpose"].view(np.uint32), err_msg=label)
    np.testing.assert_array_equal(var.view(np.uint32), g["pose_variance"].view(np.uint32), err_msg=label)
    np.testing.assert_array_equal(nt, g["n_trees"].astype(np.int32), err_msg=label)


@pytest.mark.gpu
def test_c2_full_batch_host_api(engine, c2):
    crops, g = c2
    faces = engine.analyzeFaces(list(crops), [(0, 0, CROP, CROP)] * len(crops))
    assert all(f.status == 0 for f in faces)
    pts = np.stack([f.ffd_cordinates for f in faces]).astype(np.int16)
    hp = np.array([f.headpose for f in faces], np.float32)
    var = np.array([f.pose_variance for f in faces], np.float32)
    nt = np.array([f.n_trees for f in faces], np.int32)
    _compare(pts, hp, var, nt, g, "ffd_analyze_faces")


@pytest.mark.gpu
def test_c2_full_batch_device_api(engine, c2):
    """bench.py's call: images resident in HBM, records left in HBM."""
    import torch

    import face_alignment_cvpr_2012_amd as ffd
    crops, g = c2
    n = len(crops)
    d_img = torch.from_numpy(np.ascontiguousarray(crops)).cuda()
    d_out = torch.zeros(n * ffd.FACE_RECORD_BYTES, dtype=torch.uint8, device="cuda")
    boxes = np.tile(np.array([0, 0, CROP, CROP], np.int32), (n, 1))
    engine.analyze_device(d_img.data_ptr(), CROP * CROP * 3, CROP, CROP, CROP * 3, n, boxes,
                          np.arange(n, dtype=np.int32), d_out.data_ptr())
    engine.synchronize()
    faces = ffd.faces_from_records(d_out.cpu().numpy().tobytes())
    pts = np.stack([f.ffd_cordinates for f in faces]).astype(np.int16)
    hp = np.array([f.headpose for f in faces], np.float32)
    var = np.array([f.pose_variance for f in faces], np.float32)
    nt = np.array([f.n_trees for f in faces], np.int32)
    _compare(pts, hp, var, nt, g, "ffd_analyze_faces_device")


@pytest.mark.gpu
def test_c3_bench_frame_all_faces(engine, oracle_mod):
    """bench.py --workload c3's first frame (rank 0: seed 1080), all 8 boxes."""
    from face_alignment_cvpr_2012_amd.synthetic import make_frames
    frames, boxes, _ = make_frames(1, seed=1080)
    flat = [tuple(int(v) for v in b) for b in boxes[0]]
    faces = engine.analyzeFaces([frames[0]], flat, np.zeros(len(flat), np.int32))
    assert len(flat) == 8
    for i, b in enumerate(flat):
        ref, _ = oracle_mod.analyze_face(frames[0], b, threads=8)
        np.testing.assert_array_equal(faces[i].ffd_cordinates, ref["points"], err_msg=f"box {i} {b}")
        assert np.float32(faces[i].headpose).tobytes() == np.float32(ref["headpose"]).tobytes(), i


@pytest.mark.gpu
def test_c5_bench_frame_all_faces(engine, oracle_mod):
    """bench.py --workload c5's first frame of 64 crops (rank 0: seed 5000), every face."""
    from face_alignment_cvpr_2012_amd.synthetic import make_crops
    crops, _ = make_crops(64, seed=5000)
    faces = engine.analyzeFaces(list(crops), [(0, 0, CROP, CROP)] * 64)
    for i in range(64):
        ref, _ = oracle_mod.analyze_face(crops[i], (0, 0, CROP, CROP), threads=8)
        np.testing.assert_array_equal(faces[i].ffd_cordinates, ref["points"], err_msg=f"face {i}")
        assert np.float32(faces[i].headpose).tobytes() == np.float32(ref["headpose"]).tobytes(), i


@pytest.mark.gpu
@pytest.mark.parametrize("chunk,count", [(16, 4096), (1, 256)])
def test_c2_small_batch_kernels_every_face(c2, chunk, count):
    """The small-batch kernels (k_meanshift5 / k_hp_pose1 with their ds_read_b128 component-major serial sums,
    k_votes_wg, the banded Gabor instances) on the C2 crops, in chunks of `chunk` faces, against the same
    goldens: the face-major k_meanshift variant's mismatches (DESIGN §5 tried-table) do not occur in them."""
    import face_alignment_cvpr_2012_amd as ffd
    crops, g = c2
    with ffd.FaceForest(ffd.FaceForestOptions(max_chunk_faces=chunk)) as ff:
        faces = []
        for lo in range(0, count, 256):
            faces += ff.analyzeFaces(list(crops[lo:lo + 256]), [(0, 0, CROP, CROP)] * len(crops[lo:lo + 256]))
    pts = np.stack([f.ffd_cordinates for f in faces]).astype(np.int16)
    hp = np.array([f.headpose for f in faces], np.float32)
    var = np.array([f.pose_variance for f in faces], np.float32)
    nt = np.array([f.n_trees for f in faces], np.int32)
    _compare(pts, hp, var, nt, {k: v[:count] for k, v in g.items() if k in ("points", "headpose", "pose_variance",
                                                                            "n_trees")}, f"chunks of {chunk}")
