"""The rest of the drop-in surface on the GPU, each against the CPU restatement:

* FaceForest::estimateHeadPose / estimateFacialFeatures (src/FaceForest.cpp:60-95) on an image
  sample's channels, whole sample and a sub-region (face_bbox with a non-zero origin);
* edge-case boxes the reference accepts: a face on which no head-pose patch fits (the reference
  averages 0/0: NaN head pose, trees 0..19 of forest 0, landmarks (0, 0)), W = 124 rounding, a tall
  face (125 x 375), faces taller than the whole-face Gabor staging (125 x 625, 125 x 1500); and the
  per-face statuses of the boxes it rejects;
* the multi-device entry points on the one device a box has (ffd_group_*, ffd_engine_join +
  ffd_gather_faces through RCCL);
* the engine's non-default configurations (3 x 3 patch blocks, FFD_CHANNEL_STREAMS=2, two streams, every
  face through the exact Gabor instance), read at ffd_engine_create;
* the Gabor kernels' branch-free magnitude sqrt against sqrtf for every float of its domain."""
import os

import numpy as np
import pytest

import face_alignment_cvpr_2012_amd as ffd
from conftest import crops

pytestmark = pytest.mark.gpu

EDGE_BOXES = [(30, 100, 200, 40), (5, 5, 240, 30), (100, 60, 40, 120), (61, 72, 130, 130)]


def test_estimate_headpose_and_features_match_oracle(engine, oracle_mod, fixtures):
    img, box = fixtures["images"][3], tuple(int(v) for v in fixtures["boxes"][3])
    face = engine.analyzeFace(img, box)
    tr = engine.trace(0, box[2], box[3])
    ch = tr["channels"]
    hp, var = engine.estimateHeadPose(ch)
    assert np.float32(hp) == np.float32(face.headpose) and np.float32(var) == np.float32(face.pose_variance)
    pts = engine.estimateFacialFeatures(ch, None, tr["trees"])
    assert np.array_equal(pts, np.rint(tr["ms_mean"]).astype(np.int32))  # cvRound, before the rescale
    for region in [(3, 5, 110, 115), (0, 0, 125, 125), (20, 11, 70, 90)]:
        g = engine.estimateHeadPose(ch, region)
        o = oracle_mod.estimate_headpose(ch, region)
        assert np.float32(g[0]) == np.float32(o[0]) and np.float32(g[1]) == np.float32(o[1]), region
        for trees in (tr["trees"], list(range(40, 60)), [3, 77, 12]):
            gp = engine.estimateFacialFeatures(ch, region, trees)
            op = oracle_mod.estimate_facial_features(ch, region, trees)
            assert np.array_equal(gp, op), (region, trees)


def test_estimate_rejects_bad_region(engine, fixtures):
    ch = np.zeros((38, 126, 126), np.uint32)
    with pytest.raises(ffd.FFDError):
        engine.estimateHeadPose(ch, (10, 10, 120, 120))
    with pytest.raises(ffd.FFDError):
        engine.estimateFacialFeatures(ch, None, [100])


def test_edge_boxes_match_oracle(engine, oracle_mod, fixtures):
    img = fixtures["images"][0]
    faces = engine.analyzeFaces([img], EDGE_BOXES, [0] * len(EDGE_BOXES))
    for f, box in zip(faces, EDGE_BOXES):
        ref, _ = oracle_mod.analyze_face(img, box, threads=8)
        assert f.status == 0, (box, f.status)
        assert f.n_trees == ref["n_trees"], box
        assert np.array_equal(f.ffd_cordinates, ref["points"]), box
        if np.isnan(ref["headpose"]):
            assert np.isnan(f.headpose) and np.isnan(f.pose_variance), box
            assert (f.ffd_cordinates == 0).all()
        else:
            assert np.float32(f.headpose) == np.float32(ref["headpose"]), box


def test_very_tall_faces_match_oracle(engine, oracle_mod, fixtures):
    """Scaled faces taller than MAX_FACE_H (600 rows) run through the band-staged Gabor instance
    (k_gabor_sep<..., TALL>), and faces whose integrals may reach 2^24 (255 W H >= 2^24), where the
    reference's CV_32F integral rounds, through float-accumulated integrals and the exact walker
    k_walk_fint: 125 x 1500, 125 x 625 and 125 x 3125 faces in one batch with an ordinary one."""
    img = fixtures["images"][0]
    boxes = [(100, 5, 20, 240), (61, 72, 130, 130), (40, 10, 48, 240), (120, 0, 10, 250)]
    faces = engine.analyzeFaces([img], boxes, [0] * len(boxes))
    for f, box in zip(faces, boxes):
        ref, _ = oracle_mod.analyze_face(img, box, threads=8)
        assert f.status == 0, (box, f.status)
        assert f.n_trees == ref["n_trees"], box
        assert np.array_equal(f.ffd_cordinates, ref["points"]), box
        assert np.float32(f.headpose) == np.float32(ref["headpose"]), box


def test_faces_beyond_int16_rows_match_oracle(engine, oracle_mod, fixtures):
    """No face-height limit short of memory: a 125 x 10,416 face (past round 4's 4,096-row cap) and a 125 x 37,500
    face whose vote positions leave int16 (FaceDesc::wide: VoteW lists, k_meanshift5), in one batch with an
    ordinary face (the tall ones get chunks of their own), each equal to the oracle."""
    img = np.ascontiguousarray(np.concatenate([fixtures["images"][0], fixtures["images"][1]], axis=0))
    boxes = [(120, 0, 3, 250), (61, 72, 130, 130), (120, 0, 1, 300)]
    faces = engine.analyzeFaces([img], boxes, [0] * len(boxes))
    for f, box in zip(faces, boxes):
        ref, _ = oracle_mod.analyze_face(img, box, threads=16)
        assert f.status == 0, (box, f.status)
        assert f.n_trees == ref["n_trees"], box
        assert np.array_equal(f.ffd_cordinates, ref["points"]), box
        assert np.float32(f.headpose) == np.float32(ref["headpose"]), box


def test_wide_vote_path_equals_narrow(model_path, engine, fixtures):
    """FFD_VOTES_WIDE=1 sends every face through the wide vote path (16-B VoteW lists, the k_meanshift5
    companion launch): the 20 bundled faces, as a batch and one by one, equal the ordinary path's."""
    boxes = [tuple(int(v) for v in b) for b in fixtures["boxes"]]
    want = engine.analyzeFaces(list(fixtures["images"]), boxes)
    os.environ["FFD_VOTES_WIDE"] = "1"
    try:
        wide = ffd.FaceForest(ffd.FaceForestOptions(model_path=model_path))
    finally:
        del os.environ["FFD_VOTES_WIDE"]
    try:
        got = wide.analyzeFaces(list(fixtures["images"]), boxes)
        one = [wide.analyzeFace(img, b) for img, b in zip(fixtures["images"][:3], boxes[:3])]
    finally:
        wide.close()
    for a, b in zip(got + one, want + want[:3]):
        assert np.array_equal(a.ffd_cordinates, b.ffd_cordinates) and np.float32(a.headpose) == np.float32(b.headpose)


def test_meanshift_votes_beyond_int16(engine, oracle_mod):
    """ffd_meanshift (MeanShift::shift on one list) with positions far outside int16 (a wide list) and inside
    it, equal to the oracle's restatement bit for bit; unchecked votes are skipped."""
    rng = np.random.default_rng(5)
    for centre, spread in (((40000, -70000), 30), ((120, 90), 12), ((5, 2_000_000), 8)):
        n = 700
        xy = np.stack([rng.normal(centre[0], spread, n), rng.normal(centre[1], spread, n)], 1).astype(np.int32)
        w = rng.uniform(0.1, 1.0, n).astype(np.float32)
        check = rng.uniform(size=n) < 0.9
        got = ffd.meanshift(engine, [(int(x), int(y), float(ww), bool(c)) for (x, y), ww, c in zip(xy, w, check)])
        want = oracle_mod.meanshift(xy[check], w[check])
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (centre, got, want)


def test_rejected_boxes_get_truthful_status(engine, fixtures):
    img = fixtures["images"][0]
    boxes = [(200, 200, 100, 100), (-1, 0, 50, 50), (61, 72, 130, 130), (10, 10, 200, 1)]
    faces = engine.analyzeFaces([img], boxes, [0] * len(boxes))
    assert [f.status for f in faces] == [ffd.STATUS_INVALID_ARGUMENT, ffd.STATUS_INVALID_ARGUMENT, 0,
                                        ffd.STATUS_INVALID_ARGUMENT]
    good = engine.analyzeFace(img, boxes[2])
    assert np.array_equal(faces[2].ffd_cordinates, good.ffd_cordinates)
    # a scaled face over MAX_FACE_ROWS (2^21 rows: > 50 GB of channel planes) is out of memory, not a crash
    tall = np.zeros((17000, 2, 3), np.uint8)
    f = engine.analyzeFaces([tall], [(0, 0, 1, 16800)], [0])[0]
    assert f.status == ffd.STATUS_OUT_OF_MEMORY
    assert "memory" in ffd.status_string(f.status)


def test_group_on_one_device_equals_engine(model_path, engine, fixtures):
    imgs = list(fixtures["images"][:6]) + list(crops(4, seed=3))
    boxes = [tuple(int(v) for v in b) for b in fixtures["boxes"][:6]] + [(0, 0, 150, 150)] * 4
    want = engine.analyzeFaces(imgs, boxes)
    with ffd.FaceForestGroup([0], ffd.FaceForestOptions(model_path=model_path)) as g:
        assert g.size() == 1
        got = g.analyzeFaces(imgs, boxes)
    for a, b in zip(got, want):
        assert np.array_equal(a.ffd_cordinates, b.ffd_cordinates) and a.headpose == b.headpose


def test_group_two_devices_uneven_shards(model_path, engine, fixtures):
    """ffd_group_* over 2 devices (ncclCommInitAll, image remapping per device, padded shards, one
    ncclGather, ordered D2H): 5 faces = 3 + 2, byte-for-byte equal to one engine.  Needs 2 devices."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two HIP devices")
    imgs = list(fixtures["images"][:3])
    boxes = [tuple(int(v) for v in fixtures["boxes"][i]) for i in (0, 1, 2)] + [(40, 40, 150, 150), (0, 0, 120, 130)]
    box_img = [0, 1, 2, 1, 0]
    want = engine.analyzeFaces(imgs, boxes, box_img)
    with ffd.FaceForestGroup([0, 1], ffd.FaceForestOptions(model_path=model_path)) as g:
        got = g.analyzeFaces(imgs, boxes, box_img)
    for a, b in zip(got, want):
        assert np.array_equal(a.ffd_cordinates, b.ffd_cordinates) and a.bbox == b.bbox
        assert np.float32(a.headpose).tobytes() == np.float32(b.headpose).tobytes()


def test_rccl_join_and_gather_single_rank(engine):
    import torch
    cid = ffd.comm_id()
    assert len(cid) == ffd.COMM_ID_BYTES
    engine.join(cid, 1, 0)
    assert engine.comm_info() == (1, 0)
    n = 7
    local = torch.arange(n * ffd.FACE_RECORD_BYTES, dtype=torch.int64, device="cuda").to(torch.uint8)
    root = torch.zeros_like(local)
    engine.gather(local.data_ptr(), n, root.data_ptr(), 0)
    engine.synchronize()
    assert torch.equal(local, root)


@pytest.mark.parametrize("env", [{"FFD_TRAV_G_FFD": "3", "FFD_TRAV_G_HP": "3"}, {"FFD_CHANNEL_STREAMS": "2"},
                                 {"FFD_STREAMS": "2", "FFD_CHUNK": "5"}, {"FFD_GABOR_EXACT": "1"}])
def test_engine_variants_bit_exact(model_path, oracle_mod, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        ff = ffd.FaceForest(ffd.FaceForestOptions(model_path=model_path))
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        imgs = crops(12, seed=21)
        faces = ff.analyzeFaces(list(imgs), [(0, 0, 150, 150)] * len(imgs))
        for img, f in zip(imgs, faces):
            ref, _ = oracle_mod.analyze_face(img, (0, 0, 150, 150), threads=8)
            assert np.array_equal(f.ffd_cordinates, ref["points"])
            assert np.float32(f.headpose) == np.float32(ref["headpose"])
    finally:
        ff.close()


def test_mag_sqrt_exhaustive(engine):
    """mag_sqrt (csrc/ffd_kernels.hip) == sqrtf on the device for +0 and every finite s >= 2^-96."""
    checked, bad = engine.check_mag_sqrt()
    assert checked == 1 + (0x7F800000 - 0x0F800000)
    assert bad == 0


def test_engine_closed_before_its_sample(model_path, fixtures):
    """a FaceForest closed (or its with-block left) while an ImageSample made from it lives.  The engine
    frees the sample's planes and marks it orphaned (ffd_engine_destroy); the sample's calls then fail cleanly
    and its close / garbage collection only releases host state."""
    img, box = fixtures["images"][3], tuple(int(v) for v in fixtures["boxes"][3])
    gray = np.ascontiguousarray(img[box[1]:box[1] + 100, box[0]:box[0] + 100, 1])  # any 8-bit face
    ff = ffd.FaceForest(ffd.FaceForestOptions(model_path=model_path))
    s = ffd.ImageSample(ff, gray)
    hp = s.estimateHeadPose()
    ff.close()
    with pytest.raises(ffd.FFDError, match="destroyed"):
        s.estimateHeadPose()
    with pytest.raises(ffd.FFDError):
        s.channels()
    with pytest.raises(ffd.FFDError):
        s.eval_leaves(ffd.FOREST_HEADPOSE, [(0, 0)], [0])
    s.close()
    with ffd.FaceForest(ffd.FaceForestOptions(model_path=model_path)) as ff2:
        s2 = ffd.ImageSample(ff2, gray)
        assert np.float32(s2.estimateHeadPose()[0]) == np.float32(hp[0])
    with pytest.raises(ffd.FFDError):
        s2.estimateFacialFeatures(None, list(range(20)))
    del s2  # (garbage collected after its engine: host state only)
