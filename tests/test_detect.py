"""Haar face detector (FaceForest::detectFace, /root/reference/src/FaceForest.cpp
:136-159), CPU side: the converted cascade against the reference's XML, and the restatement
(oracle/ffd_oracle.cpp haar_scan / haar_group / widen_box) against its committed goldens and a
sanity band.  Parity with OpenCV's detectMultiScale is UNPINNED (OpenCV is not in this image and
the reference ships no detections); the GPU detector is compared with this restatement bit for bit
in tests/test_gpu_detect.py."""
import json
import os
import xml.etree.ElementTree as ET

import numpy as np
import pytest

from face_alignment_cvpr_2012_amd import model as fmodel
from face_alignment_cvpr_2012_amd import synthetic

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFERENCE = os.environ.get("FFD_REFERENCE", "/root/reference")
GOLDEN = json.load(open(os.path.join(REPO, "tests", "golden", "detect_golden.json")))
# maxWeakCount of the 22 stages of data/haarcascade_frontalface_alt.xml
STAGE_SIZES = [3, 16, 21, 39, 33, 44, 50, 51, 56, 71, 80, 103, 111, 102, 135, 137, 140, 160, 177, 182, 211, 213]


def test_cascade_known_answers(model_path):
    m = fmodel.load(model_path)
    assert m["haar.window"].tolist() == [20, 20]
    assert m["haar.stage_ntrees"].tolist() == STAGE_SIZES
    assert m["haar.stage_first"].tolist() == np.concatenate([[0], np.cumsum(STAGE_SIZES)[:-1]]).tolist()
    assert m["haar.weak_feature"].shape == (2135,) and m["haar.feature_rect"].shape == (2135, 3, 4)
    # first weak classifier / feature of the file (stage 0, tree 0)
    assert m["haar.weak_feature"][0] == 0
    assert m["haar.weak_threshold"][0] == np.float32(4.0141958743333817e-03)
    assert m["haar.weak_leaves"][0].tolist() == [np.float32(3.3794190734624863e-02), np.float32(8.3781069517135620e-01)]
    assert m["haar.feature_rect"][0].tolist() == [[3, 7, 14, 4], [3, 9, 14, 2], [0, 0, 0, 0]]
    assert m["haar.feature_weight"][0].tolist() == [-1.0, 2.0, 0.0]
    assert m["haar.stage_threshold"][0] == np.float32(8.2268941402435303e-01)


@pytest.mark.reference
def test_cascade_matches_independent_xml_parse(model_path):
    path = os.path.join(REFERENCE, "data", "haarcascade_frontalface_alt.xml")
    if not os.path.exists(path):
        pytest.skip("reference tree not present")
    root = ET.parse(path).getroot().find("cascade")
    m = fmodel.load(model_path)
    thr, feat, wthr, leaves = [], [], [], []
    for st in root.find("stages"):
        thr.append(np.float32(float(st.find("stageThreshold").text)))
        for wc in st.find("weakClassifiers"):
            nd = wc.find("internalNodes").text.split()
            feat.append(int(nd[2]))
            wthr.append(np.float32(float(nd[3])))
            leaves.append([np.float32(float(v)) for v in wc.find("leafValues").text.split()])
    rects, weights = [], []
    for f in root.find("features"):
        r = [[int(float(v)) for v in e.text.split()[:4]] for e in f.find("rects")]
        w = [np.float32(float(e.text.split()[4])) for e in f.find("rects")]
        rects.append(r + [[0, 0, 0, 0]] * (3 - len(r)))
        weights.append(w + [np.float32(0)] * (3 - len(w)))
    assert np.array_equal(m["haar.stage_threshold"], np.array(thr, np.float32))
    assert np.array_equal(m["haar.weak_feature"], np.array(feat))
    assert np.array_equal(m["haar.weak_threshold"], np.array(wthr, np.float32))
    assert np.array_equal(m["haar.weak_leaves"], np.array(leaves, np.float32))
    assert np.array_equal(m["haar.feature_rect"], np.array(rects))
    assert np.array_equal(m["haar.feature_weight"], np.array(weights, np.float32))


def _iou(a, b):
    x0, y0 = max(a[0], b[0]), max(a[1], b[1])
    x1, y1 = min(a[0] + a[2], b[0] + b[2]), min(a[1] + a[3], b[1] + b[3])
    i = max(0, x1 - x0) * max(0, y1 - y0)
    return i / (a[2] * a[3] + b[2] * b[3] - i)


def test_oracle_detects_every_bundled_face(oracle_mod, fixtures):
    """Sanity band: one detection per bundled LFW image, overlapping its annotated box."""
    for i, img in enumerate(fixtures["images"]):
        det = oracle_mod.detect_faces(img, widen=False)
        assert len(det) == 1, (i, det)
        assert _iou(fixtures["boxes"][i], det[0]) > 0.55, (i, det, fixtures["boxes"][i])


def test_oracle_goldens(oracle_mod, fixtures):
    for i, img in enumerate(fixtures["images"]):
        boxes, raw = oracle_mod.detect_faces(img, raw=True)
        assert boxes.tolist() == GOLDEN["fixtures"][i]["boxes"], i
        assert len(raw) == GOLDEN["fixtures"][i]["n_raw"], i


def test_oracle_frames_goldens_and_paste_boxes(oracle_mod):
    frames, boxes, paste = synthetic.make_frames(2)
    for k, fr in enumerate(frames):
        det, raw = oracle_mod.detect_faces(fr, raw=True)
        g = GOLDEN["frames"][k]
        assert det.tolist() == g["boxes"] and len(raw) == g["n_raw"] and raw[:16].tolist() == g["raw_head"]
        # every pasted face found (widened detection vs the widened paste box)
        for b in boxes[k]:
            assert max(_iou(b, d) for d in det) > 0.5, (k, b)


def test_oracle_option_semantics(oracle_mod, fixtures):
    img = fixtures["images"][3]
    boxes, raw = oracle_mod.detect_faces(img, raw=True)
    # min_neighbors 0: groupRectangles returns the candidates unchanged
    ungrouped = oracle_mod.detect_faces(img, min_neighbors=0, widen=False)
    assert np.array_equal(ungrouped, raw)
    # widen: detectFace's enlargement of the grouped boxes
    tight = oracle_mod.detect_faces(img, widen=False)
    h, w = img.shape[:2]
    assert [list(synthetic.face_box_from_detection(b, w, h)) for b in tight] == boxes.tolist()
    # min_size above every window: nothing scanned
    assert len(oracle_mod.detect_faces(img, min_size=400)) == 0
    # a frame smaller than the cascade window
    assert len(oracle_mod.detect_faces(np.zeros((15, 15, 3), np.uint8))) == 0
