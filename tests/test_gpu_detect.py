"""Haar face detector on the GPU (face_alignment_cvpr_2012_amd/csrc/ffd_haar.hip) vs the CPU
restatement (oracle/ffd_oracle.cpp), bit-exact: the ungrouped detectMultiScale candidates in scan
order, the grouped + widened detectFace boxes, the option variants, multi-frame batches of mixed
sizes, the device-resident entry point and analyzeImage end to end (SURVEY.md §8(f) #1;
/root/reference/src/FaceForest.cpp:136-181).  Parity with OpenCV itself is unpinned."""
import ctypes

import numpy as np
import pytest

import face_alignment_cvpr_2012_amd as ffd
from face_alignment_cvpr_2012_amd import synthetic

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frames():
    fr, boxes, _ = synthetic.make_frames(2)
    return fr, boxes


def test_candidates_and_boxes_fixtures(engine, oracle_mod, fixtures):
    for i, img in enumerate(fixtures["images"]):
        want_boxes, want_raw = oracle_mod.detect_faces(img, raw=True)
        raw = engine.detect_candidates(img)
        assert np.array_equal(raw, want_raw), i
        assert np.array_equal(engine.detectFace(img), want_boxes), i


def test_1080p_frames_batch(engine, oracle_mod, frames):
    fr, boxes = frames
    got = engine.detectFaces(list(fr))
    for k in range(len(fr)):
        want, want_raw = oracle_mod.detect_faces(fr[k], raw=True)
        assert np.array_equal(got[k], want), k
        assert np.array_equal(engine.detect_candidates(fr[k]), want_raw), k
        assert len(want) >= len(boxes[k])


def test_options(engine, oracle_mod, fixtures, frames):
    img = frames[0][1]
    for opt in (ffd.FaceDetectionOption(min_neighbors=0, widen=False),
                ffd.FaceDetectionOption(min_neighbors=3),
                ffd.FaceDetectionOption(min_feature_size=60, search_scale_factor=1.1),
                ffd.FaceDetectionOption(min_feature_size=20, search_scale_factor=1.25, widen=False)):
        want = oracle_mod.detect_faces(img, min_size=opt.min_feature_size, min_neighbors=opt.min_neighbors,
                                       scale_factor=opt.search_scale_factor, widen=opt.widen)
        assert np.array_equal(engine.detectFace(img, opt), want), opt


def test_mixed_sizes_and_edge_frames(engine, oracle_mod, fixtures):
    rng = np.random.default_rng(5)
    imgs = [fixtures["images"][0], np.zeros((15, 15, 3), np.uint8),  # smaller than the window
            rng.integers(0, 256, (240, 320, 3), dtype=np.uint8),      # noise
            np.ascontiguousarray(fixtures["images"][4][:, ::-1]),      # mirrored face
            np.full((64, 90, 3), 128, np.uint8)]                      # flat
    got = engine.detectFaces(imgs)
    for k, img in enumerate(imgs):
        assert np.array_equal(got[k], oracle_mod.detect_faces(img)), k


def test_device_entry_point(engine, oracle_mod, frames):
    import torch
    fr = frames[0]
    d = torch.from_numpy(np.ascontiguousarray(fr)).cuda()
    n_img, h, w = fr.shape[:3]
    cap = 256
    boxes = np.zeros((cap, 4), np.int32)
    owner = np.zeros(cap, np.int32)
    n = ctypes.c_int32()
    opt = ffd._det_opt(None)
    st = ffd.lib().ffd_detect_faces_device(engine.handle, ctypes.c_void_p(d.data_ptr()), h * w * 3, w, h, w * 3,
                                           n_img, ctypes.byref(opt), boxes.ctypes.data, owner.ctypes.data, cap,
                                           ctypes.byref(n))
    assert st == 0
    for k in range(n_img):
        assert np.array_equal(boxes[: n.value][owner[: n.value] == k], oracle_mod.detect_faces(fr[k])), k


def test_analyze_image_end_to_end(engine, oracle_mod, fixtures, frames):
    """analyzeImage(img): GPU detection then analyzeFace on every box == oracle detect + analyze."""
    for img in (fixtures["images"][2], frames[0][0]):
        faces = engine.analyzeImage(img)
        want = oracle_mod.detect_faces(img)
        assert [f.bbox for f in faces] == [tuple(b) for b in want.tolist()]
        for f, b in zip(faces, want):
            ref, _ = oracle_mod.analyze_face(img, tuple(int(v) for v in b), threads=8)
            assert f.status == 0
            assert np.array_equal(f.ffd_cordinates, ref["points"])
            assert np.float32(f.headpose) == np.float32(ref["headpose"])


@pytest.mark.parametrize("rerun_cap", ["0", "16384"])
def test_frames_over_the_candidate_capacity(engine, oracle_mod, frames, fixtures, monkeypatch, rerun_cap):
    """A frame with more raw detections than the grouping holds (8,192 per frame; detectMultiScale has no
    limit, FaceForest.cpp:146) is run again on its own with a capacity that holds them all, its neighbours in
    the batch unaffected.  Forced here with a capacity of 64 (FFD_DETECT_CAP); with FFD_DETECT_RERUN_CAP=16384
    the re-run groups with its component labels in global memory (k_haar_group<true>)."""
    fr, _ = frames
    imgs = [fr[0], fixtures["images"][3], fr[1], fixtures["images"][8]]
    want = [oracle_mod.detect_faces(im) for im in imgs]
    raws = [len(oracle_mod.detect_faces(im, raw=True)[1]) for im in imgs]
    assert max(raws) > 64 and min(raws) <= 64 or max(raws) > 64  # at least one frame overflows
    monkeypatch.setenv("FFD_DETECT_CAP", "64")
    monkeypatch.setenv("FFD_DETECT_RERUN_CAP", rerun_cap)
    got = engine.detectFaces(imgs)
    for k in range(len(imgs)):
        assert np.array_equal(got[k], want[k]), (k, raws[k])
    assert np.array_equal(engine.detect_candidates(fr[0]), oracle_mod.detect_faces(fr[0], raw=True)[1])


def tiled_frame(fixtures, oracle_mod, size, h, w):
    """A frame tiled with one bundled face scaled to size x size: tens of thousands of raw detections."""
    img = fixtures["images"][0]
    b = [int(v) for v in fixtures["boxes"][0]]
    face = np.ascontiguousarray(img[b[1]:b[1] + b[3], b[0]:b[0] + b[2]])
    f = np.stack([oracle_mod.resize(np.ascontiguousarray(face[:, :, c]), size, size) for c in range(3)], 2)
    return np.ascontiguousarray(np.tile(f, (h // size + 1, w // size + 1, 1))[:h, :w])


def test_crowded_frame_tens_of_thousands_of_candidates(engine, oracle_mod, fixtures):
    """A 3840 x 2160 frame tiled with 40-px faces gives ~4 x 10^4 raw detections, far past the grouping's LDS
    capacity (8,192): the frame is re-run with its component labels in global memory, labelled by the
    multi-workgroup min-label rounds (k_haar_label_round / k_haar_label_jump); boxes and candidates equal the
    restatement's (the large-N re-run measured, not only the forced small capacity)."""
    import time
    frame = tiled_frame(fixtures, oracle_mod, 40, 2160, 3840)
    want, want_raw = oracle_mod.detect_faces(frame, raw=True)
    assert len(want_raw) > 4 * 8192
    engine.detectFaces([frame])  # warm
    t = time.perf_counter()
    got = engine.detectFaces([frame])[0]
    ms = (time.perf_counter() - t) * 1e3
    print(f"crowded 4K frame: {len(want_raw)} raw candidates, {len(want)} boxes, {ms:.1f} ms")
    assert np.array_equal(got, want)
    assert np.array_equal(engine.detect_candidates(frame), want_raw)
