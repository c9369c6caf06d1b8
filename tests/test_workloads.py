"""BASELINE.json's other configs as parity cases: C3 1080p frames with several
detectFace-enlarged boxes per frame (125 x ~148 faces), C5-style many-faces-per-image batches."""
import numpy as np
import pytest

from face_alignment_cvpr_2012_amd.synthetic import face_box_from_detection, make_frames


def test_detect_face_enlargement_rule():
    # FaceForest.cpp:148-158: offsets int(w*0.05) / int(w*0.15), then intersect with the image
    assert face_box_from_detection((100, 50, 100, 100), 640, 480) == (95, 50, 110, 130)
    assert face_box_from_detection((0, 0, 61, 61), 640, 480) == (0, 0, 64, 79)      # clipped left
    assert face_box_from_detection((600, 400, 100, 100), 640, 480) == (595, 400, 45, 80)
    assert face_box_from_detection((700, 10, 20, 20), 640, 480) == (0, 0, 0, 0)      # outside


def test_frames_are_deterministic_and_boxes_fit():
    f1, b1, p1 = make_frames(1, seed=5)
    f2, b2, p2 = make_frames(1, seed=5)
    assert np.array_equal(f1, f2) and np.array_equal(b1, b2)
    x, y, w, h = b1[0].T
    assert (x >= 0).all() and (y >= 0).all() and (x + w <= 1920).all() and (y + h <= 1080).all()
    assert ((h / w) > 1.1).all()  # Haar-like: taller than wide after enlargement


def test_c3_geometry_matches_oracle(oracle_mod):
    _, boxes, _ = make_frames(1, seed=6)
    for b in boxes[0]:
        fw, fh, nhp, nmp = oracle_mod.geometry(int(b[2]), int(b[3]))
        assert fw in (124, 125) and 140 <= fh <= 160  # int(cols * (125.f / cols)) may round down
        assert nmp == -(-(fw - 31) // 3) * -(-(fh - 31) // 3)  # grid x, y in [0, size - 31) step 3 (face_utils.cpp:255-265)


@pytest.mark.gpu
def test_c3_frames_bit_exact(engine, oracle_mod):
    frames, boxes, _ = make_frames(2, seed=7)
    flat = [tuple(int(v) for v in b) for fb in boxes for b in fb]
    box_img = np.repeat(np.arange(len(frames)), boxes.shape[1]).astype(np.int32)
    faces = engine.analyzeFaces(list(frames), flat, box_img)
    for i, (b, k) in enumerate(zip(flat, box_img)):
        ref, rt = oracle_mod.analyze_face(frames[k], b, threads=8, trace=True)
        tr = engine.trace(i, b[2], b[3])
        np.testing.assert_array_equal(tr["hp_leaves"], rt["hp_leaves"], err_msg=f"face {i}")
        np.testing.assert_array_equal(tr["mp_leaves"], rt["mp_leaves"], err_msg=f"face {i}")
        assert np.array_equal(faces[i].ffd_cordinates, ref["points"]), i
        assert np.float32(faces[i].headpose) == np.float32(ref["headpose"]), i


@pytest.mark.gpu
def test_many_faces_per_image(engine, oracle_mod, fixtures):
    # C5 shape: many boxes on one image in one batch (here 64 jittered boxes on one fixture)
    img = fixtures["images"][3]
    x, y, w, h = (int(v) for v in fixtures["boxes"][3])
    rng = np.random.default_rng(64)
    boxes = []
    for _ in range(64):
        dx, dy, dw = (int(v) for v in rng.integers(-8, 9, size=3))
        boxes.append((max(0, x + dx), max(0, y + dy), w + dw, w + dw))
    faces = engine.analyzeFaces([img], boxes, np.zeros(64, np.int32))
    for i in range(64):
        ref, _ = oracle_mod.analyze_face(img, boxes[i], threads=8)
        assert np.array_equal(faces[i].ffd_cordinates, ref["points"]), i
        assert np.float32(faces[i].headpose).tobytes() == np.float32(ref["headpose"]).tobytes(), i


@pytest.mark.gpu
def test_c4_density_grid_bit_exact(model_path, oracle_mod, fixtures):
    """C4's 4x patch density: FFD grid step (x=2, y=1) -> 47 x 94 = 4,418 patches per 125x125 face."""
    import face_alignment_cvpr_2012_amd as ffd
    opts = ffd.FaceForestOptions(model_path=model_path,
                                 mp_option=ffd.MultiPartEstimatorOption(step_size=2, step_size_y=1))
    imgs = [fixtures["images"][i] for i in (0, 5, 11)]
    boxes = [tuple(int(v) for v in fixtures["boxes"][i]) for i in (0, 5, 11)]
    with ffd.FaceForest(opts) as ff:
        assert ff.geometry(150, 150)[3] == 47 * 94
        faces = ff.analyzeFaces(imgs, boxes)
        traces = [ff.trace(i, b[2], b[3]) for i, b in enumerate(boxes)]
    oracle_mod.set_steps(4, 2, 1)
    try:
        for i, (img, b) in enumerate(zip(imgs, boxes)):
            ref, rt = oracle_mod.analyze_face(img, b, threads=8, trace=True)
            np.testing.assert_array_equal(traces[i]["mp_leaves"], rt["mp_leaves"], err_msg=f"face {i}")
            np.testing.assert_array_equal(traces[i]["vote_counts"], rt["vote_counts"])
            assert np.array_equal(faces[i].ffd_cordinates, ref["points"]), i
    finally:
        oracle_mod.set_steps(4, 3, 3)


def _synth_forest(tmp_path, depth, trees=20):
    import subprocess
    from conftest import REPO, MODEL
    out = tmp_path / f"c4_d{depth}.bin"
    exe = f"{REPO}/face_alignment_cvpr_2012_amd/bin/ffd_synth_forest"
    subprocess.run([exe, MODEL, str(out), str(depth), str(trees), "4"], check=True, capture_output=True)
    return str(out)


def test_c4_synthetic_forest_structure(tmp_path):
    from face_alignment_cvpr_2012_amd import model as fm
    path = _synth_forest(tmp_path, 6, trees=3)
    m = fm.load(path)
    assert list(m["mp.param"][[0, 3, 7]]) == [6, 3, 1]
    off = m["mp.tree_node_off"]
    assert off[-1] == 3 * (2 ** 7 - 1) and m["mp.leaf_n"].size == 3 * 2 ** 6
    leaf = m["mp.node_leaf"][off[0]:off[1]]
    assert leaf[0] == -1 and (leaf >= 0).sum() == 64  # complete: 63 splits, 64 leaves (pre-order)
    sp = m["mp.node_split"][m["mp.node_leaf"] < 0]
    assert sp[:, 0].max() <= 37 and sp[:, [3, 4, 7, 8]].min() >= 1 and sp[:, [3, 4, 7, 8]].max() <= 22
    assert (sp[:, 1] + sp[:, 3]).max() <= 30 and (sp[:, 2] + sp[:, 4]).max() <= 30


@pytest.mark.gpu
def test_c4_deep_synthetic_forest_bit_exact(tmp_path, fixtures):
    """C4: one synthetic forest of 20 complete trees for every pose bin, 4x patch density."""
    import face_alignment_cvpr_2012_amd as ffd
    import oracle
    path = _synth_forest(tmp_path, 12)
    opts = ffd.FaceForestOptions(model_path=path, mp_option=ffd.MultiPartEstimatorOption(step_size=2, step_size_y=1))
    idx = (2, 9)
    imgs = [fixtures["images"][i] for i in idx]
    boxes = [tuple(int(v) for v in fixtures["boxes"][i]) for i in idx]
    with ffd.FaceForest(opts) as ff:
        faces = ff.analyzeFaces(imgs, boxes)
        traces = [ff.trace(i, b[2], b[3]) for i, b in enumerate(boxes)]
    oracle.load_model(path)
    oracle.set_steps(4, 2, 1)
    try:
        for i, (img, b) in enumerate(zip(imgs, boxes)):
            ref, rt = oracle.analyze_face(img, b, threads=8, trace=True)
            assert faces[i].n_trees == 20
            np.testing.assert_array_equal(traces[i]["mp_leaves"], rt["mp_leaves"], err_msg=f"face {i}")
            assert np.array_equal(faces[i].ffd_cordinates, ref["points"]), i
    finally:
        oracle.set_steps(4, 3, 3)
        from conftest import MODEL
        oracle.load_model(MODEL)


@pytest.mark.gpu
def test_c4_depth20_forest_bit_exact(tmp_path, fixtures):
    """C4 as BASELINE.json states it: 20 complete trees of depth 20 (42 M nodes, 21 M leaves) for
    every pose bin, at 4x patch density: leaf ordinals and landmarks against the oracle on one face.
    The depth-20 trees also exercise the traversal's far child offsets (subtrees > 65535 pairs)."""
    import face_alignment_cvpr_2012_amd as ffd
    import oracle
    path = _synth_forest(tmp_path, 20)
    opts = ffd.FaceForestOptions(model_path=path, mp_option=ffd.MultiPartEstimatorOption(step_size=2, step_size_y=1))
    img, b = fixtures["images"][4], tuple(int(v) for v in fixtures["boxes"][4])
    with ffd.FaceForest(opts) as ff:
        face = ff.analyzeFace(img, b)
        tr = ff.trace(0, b[2], b[3])
    oracle.load_model(path)
    oracle.set_steps(4, 2, 1)
    try:
        ref, rt = oracle.analyze_face(img, b, threads=16, trace=True)
        assert face.n_trees == 20 and tr["mp_leaves"].shape == rt["mp_leaves"].shape
        np.testing.assert_array_equal(tr["mp_leaves"], rt["mp_leaves"])
        assert np.array_equal(face.ffd_cordinates, ref["points"])
    finally:
        oracle.set_steps(4, 3, 3)
        from conftest import MODEL
        oracle.load_model(MODEL)
