"""eval_ffd end to end: config / annotation readers, the pose-bucketed 90 / 10 split
and evalForest over an annotation file plus images (face_alignment_cvpr_2012_amd/config.py, eval.py).

Fixtures: tests/golden/index_random_subset.txt and tests/golden/config_ffd.txt are verbatim copies of the
reference's data files (data/imgs/index_random_subset.txt, data/config_ffd.txt); the images are the
pre-decoded tests/golden/faces.npz.  Expected landmarks come from the oracle goldens
(tests/golden/oracle_golden.npz, fixtures 0..19 in file order)."""
import os

import numpy as np
import pytest

from face_alignment_cvpr_2012_amd import config
from face_alignment_cvpr_2012_amd import eval as fe

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ANN = os.path.join(GOLDEN, "index_random_subset.txt")
# the split eval_ffd.cpp:158-169 makes of the bundled file: buckets (pose -2..2) of 4 / 1 / 7 / 1 / 7
# annotations keep int(n * 0.9f) = 3 / 0 / 6 / 0 / 6 for training; the last of each bucket tests
TEST_SPLIT = ["George_HW_Bush_0008.jpg", "Elton_John_0001.jpg", "Bono_0002.jpg", "Dick_Vermeil_0002.jpg",
              "Laura_Bush_0008.jpg"]


def _golden():
    return np.load(os.path.join(GOLDEN, "oracle_golden.npz"))


def test_annotations_match_fixtures(fixtures):
    ok, anns = config.load_annotations(ANN)
    assert ok and len(anns) == 20
    assert [a.url for a in anns] == [str(n) for n in fixtures["names"]]
    assert np.array_equal(np.array([a.bbox for a in anns]), fixtures["boxes"])
    assert np.array_equal(np.array([a.pose for a in anns]), fixtures["poses"])
    assert np.array_equal(np.stack([a.parts for a in anns]), fixtures["parts"])
    assert config.load_annotations(ANN + ".missing") == (False, [])


def test_annotation_grammar():
    text = "# comment line\na.jpg 1 2 3 4 -1 2 5 6 7 8 \nb.jpg 0 0 10 10 0 0\n"
    a = config.parse_annotations(text)
    assert [x.url for x in a] == ["a.jpg", "b.jpg"]
    assert a[0].bbox == (1, 2, 3, 4) and a[0].pose == -1 and a[0].parts.tolist() == [[5, 6], [7, 8]]
    assert a[1].parts.shape == (0, 2)
    with pytest.raises(ValueError):  # boost::split on " ": a double space is an empty field
        config.parse_annotations("a.jpg 1  2 3 4 0 0\n")


def test_split_membership():
    _, anns = config.load_annotations(ANN)
    train, test = config.split_by_pose(anns)
    assert [len(b) for b in train] == [3, 0, 6, 0, 6]
    assert [a.url for b in test for a in b] == TEST_SPLIT
    # every bucket keeps its file order; train + test is the bucket
    for tr, te in zip(train, test):
        assert all(a.pose == (tr + te)[0].pose for a in tr + te)
    # int(size * 0.9f) in float: 10 -> 9, 20 -> 18, 1 -> 0, 1326 faces' buckets never round up past size
    for n in (1, 2, 9, 10, 11, 20, 29, 30, 100, 663, 1000):
        anns_n = [config.FaceAnnotation(f"{i}", (0, 0, 1, 1), 0, np.zeros((10, 2), np.int32)) for i in range(n)]
        tr, te = config.split_by_pose(anns_n)
        assert len(tr[2]) == int(np.float32(n) * np.float32(0.9)) and len(tr[2]) + len(te[2]) == n
    with pytest.raises(IndexError):
        config.split_by_pose([config.FaceAnnotation("x", (0, 0, 1, 1), 3, np.zeros((10, 2), np.int32))])


def test_config_file():
    ok, p = config.load_config_file(os.path.join(GOLDEN, "config_ffd.txt"))
    assert ok
    assert (p.image_path, p.tree_path, p.ntrees, p.ntests, p.max_depth, p.min_patches, p.nimages, p.npatches,
            p.face_size, p.features) == ("../../database/faces/lfw/lfw_ffd_ann.txt", "data/trees_ffd", 20, 2500, 20,
                                         20, 600, 150, 125, [0, 1, 2])
    assert p.patch_size_ratio == np.float32(0.25) and p.getPatchSize() == 31
    ok, d = config.load_config_file(os.path.join(GOLDEN, "no_such_config.txt"))
    assert not ok and (d.max_depth, d.ntests, d.ntrees, d.face_size) == (15, 250, 10, 100)


def test_intersect_and_enlarge_face():
    assert config.intersect((-5, -5, 20, 20), (0, 0, 10, 10)) == (0, 0, 10, 10)
    assert config.intersect((20, 20, 5, 5), (0, 0, 10, 10)) == (0, 0, 0, 0)
    ann = config.FaceAnnotation("x", (61, 72, 130, 130), 2, np.array([[36, 46], [53, 43]], np.int32))
    box, a2 = config.enlarge_face((250, 250, 3), ann)
    assert box == (48, 59, 156, 156) and a2.bbox == (0, 0, 156, 156)  # offset (13, 13)
    assert a2.parts.tolist() == [[49, 59], [66, 56]]
    box, _ = config.enlarge_face((200, 200, 3), config.FaceAnnotation("y", (150, 150, 49, 49), 0, np.zeros((0, 2))))
    assert box == (146, 146, 54, 54)  # clipped to the image


def test_image_store(tmp_path, fixtures):
    store = config.ImageStore(arrays=os.path.join(GOLDEN, "faces.npz"))
    assert np.array_equal(store("Bob_Beauprez_0001.jpg"), fixtures["images"][0])
    np.save(tmp_path / "a.png.npy", fixtures["images"][1])
    s2 = config.ImageStore(str(tmp_path) + "/")
    assert np.array_equal(s2("a.png"), fixtures["images"][1])
    assert s2("missing.jpg") is None
    pil = pytest.importorskip("PIL.Image")
    pil.fromarray(np.ascontiguousarray(fixtures["images"][2][:, :, ::-1])).save(tmp_path / "c.png")
    assert np.array_equal(s2("c.png"), fixtures["images"][2])  # lossless: BGR order restored


class _GoldenAnalyzer:
    """analyzeFace from the oracle goldens (landmarks of fixture k for its annotated box)."""

    def __init__(self, fixtures):
        g = _golden()
        self.by_box = {}
        for k in range(20):
            key = (fixtures["images"][k].tobytes()[:4096], tuple(int(v) for v in fixtures["boxes"][k]))
            self.by_box[key] = g["points"][k]

    def analyzeFace(self, img, bbox):
        from face_alignment_cvpr_2012_amd import Face
        pts = self.by_box[(np.ascontiguousarray(img).tobytes()[:4096], tuple(bbox))]
        return Face(headpose=0.0, bbox=bbox, ffd_cordinates=pts)


def test_eval_forest_split_and_errors_txt(tmp_path, fixtures):
    out = tmp_path / "output" / "errors.txt"
    store = config.ImageStore(arrays=os.path.join(GOLDEN, "faces.npz"))
    errors, done = fe.run_eval(_GoldenAnalyzer(fixtures), ANN, store, out_path=str(out))
    assert [a.url for a in done] == TEST_SPLIT
    names = [str(n) for n in fixtures["names"]]
    g = _golden()
    want = [fe.landmark_errors(fixtures["parts"][names.index(u)], g["points"][names.index(u)]) for u in TEST_SPLIT]
    assert np.array_equal(np.array(errors), np.array(want))
    text = out.read_text()
    assert text == fe.format_errors(want)
    lines = text.splitlines(True)
    assert len(lines) == 5 and all(line.endswith(" \n") and len(line.split()) == 10 for line in lines)


def test_eval_forest_skips_missing_images(fixtures):
    store = config.ImageStore(arrays={str(n): im for n, im in zip(fixtures["names"], fixtures["images"])
                                      if str(n) != "Bono_0002.jpg"})
    logged = []
    _, anns = config.load_annotations(ANN)
    _, test = config.split_by_pose(anns)
    errors, done = fe.eval_forest(_GoldenAnalyzer(fixtures), test, store, log=logged.append)
    assert [a.url for a in done] == [u for u in TEST_SPLIT if u != "Bono_0002.jpg"]
    assert len(errors) == 4 and logged == ["Could not load: Bono_0002.jpg"]


@pytest.mark.gpu
def test_engine_eval_ffd_split(tmp_path, capsys, fixtures):
    """The engine through eval_ffd's path on the bundled annotation file: the 5 test faces' errors equal
    the oracle goldens' (landmarks bit-exact), and errors.txt has the reference's format."""
    out = tmp_path / "errors.txt"
    assert fe.main(["--out", str(out)]) == 0
    names = [str(n) for n in fixtures["names"]]
    g = _golden()
    want = [fe.landmark_errors(fixtures["parts"][names.index(u)], g["points"][names.index(u)]) for u in TEST_SPLIT]
    assert out.read_text() == fe.format_errors(want)
    assert "mean IOD error" in capsys.readouterr().out
