"""The C++ drop-in from a reference source's point of view (VERDICT r4 "next" #1): tests/cxx/reference_includes.cpp
includes exactly the reference's header set of src/eval_ffd.cpp:11-13 and src/demo.cpp:11-16 (<FaceForest.hpp>,
<Constants.hpp>, <face_utils.hpp>, <Tree.hpp>, <ImageSample.hpp>, <MPSample.hpp>; trace.hpp / Viewer.hpp are the
reference's logging and UI) with no #define, and uses every symbol of those headers that eval_ffd and demo use:
eval_ffd's main and evalForest (errors.txt), demo's analyzeImage and trainTree (Tree<MPSample>(samples, param, &rng,
path) over MPSample's training constructor), the static FaceForest::detectFace with a CascadeClassifier loaded by
the caller.

CPU: the program compiles against the forwarding headers and its host-only pieces (readers, split, loadImage,
enlargeFace, ROI, norm, cvRound scaling, areaUnderCurve, constants, an uninitialised FaceForest) equal the Python
restatements.  GPU: eval_ffd's errors.txt equals the oracle goldens' (the split's 5 faces); detectFace runs the
classifier it is given — the bundled cascade and a second one (its first 12 stages) each equal the CPU
restatement of that cascade, and differ from each other; the trained tree equals the engine trainer's byte for
byte."""
import os
import re
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
SRC = os.path.join(REPO, "tests", "cxx", "reference_includes.cpp")
LIB = os.path.join(REPO, "face_alignment_cvpr_2012_amd", "lib")
ANN = os.path.join(GOLDEN, "index_random_subset.txt")
TEST_SPLIT = ["George_HW_Bush_0008.jpg", "Elton_John_0001.jpg", "Bono_0002.jpg", "Dick_Vermeil_0002.jpg",
              "Laura_Bush_0008.jpg"]


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    if not os.path.exists(os.path.join(LIB, "libffd.so")):
        pytest.skip("libffd.so not built (make)")
    src = open(SRC).read()
    includes = re.findall(r"^#include <(\w+\.hpp)>", src, re.M)
    assert includes == ["FaceForest.hpp", "Constants.hpp", "face_utils.hpp", "Tree.hpp", "ImageSample.hpp", "MPSample.hpp"]
    assert not re.search(r"^\s*#\s*define", src, re.M)
    out = str(tmp_path_factory.mktemp("ri") / "reference_includes")
    r = subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Werror", "-I" + os.path.join(REPO, "include"), SRC, "-o",
                        out, "-L" + LIB, "-lffd", "-Wl,-rpath," + LIB], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


def write_ppm(path, bgr):
    h, w = bgr.shape[:2]
    with open(path, "wb") as f:
        f.write(b"P6\n# BGR fixture written as RGB\n%d %d\n255\n" % (w, h))
        f.write(np.ascontiguousarray(bgr[:, :, ::-1]).tobytes())


@pytest.fixture(scope="module")
def image_dir(tmp_path_factory, fixtures):
    """The 20 bundled faces as PPM files under their annotation names, with a copy of the annotation file."""
    d = tmp_path_factory.mktemp("imgs")
    for name, img in zip(fixtures["names"], fixtures["images"]):
        write_ppm(d / str(name), img)
    (d / "index.txt").write_text(open(ANN).read())
    return d


def _run(exe, *args, cwd=None, env=None, timeout=600):
    return subprocess.run([exe] + [str(a) for a in args], capture_output=True, text=True, timeout=timeout, cwd=cwd,
                          env=env)


def test_host_pieces(exe, image_dir, fixtures):
    from face_alignment_cvpr_2012_amd import config
    r = _run(exe, "cpu", image_dir / "index.txt", image_dir / str(fixtures["names"][0]),
             os.path.join(GOLDEN, "config_ffd.txt"))
    assert r.returncode == 0, r.stderr
    out = dict(line.split(" ", 1) for line in r.stdout.strip().splitlines())
    assert out["config"] == "1 data/trees_ffd 20 125 31"
    assert out["annotations"] == "1 20"
    assert out["test_split"].split() == TEST_SPLIT
    img = fixtures["images"][0]
    h, w = img.shape[:2]
    assert out["image"].split() == ["1", str(h), str(w), "3", str(img[0, 0, 0]), str(img[-1, -1, 2])]
    _, anns = config.load_annotations(ANN)
    box, a2 = config.enlarge_face(img.shape, anns[0])
    assert [int(v) for v in out["enlarge"].split()] == list(box) + list(a2.parts[0])
    assert [int(v) for v in out["roi"].split()] == [box[3], box[2], int(img[box[1], box[0], 0])]
    p = anns[0].parts
    left, right = (p[0] + p[1]) / np.float32(2), (p[6] + p[7]) / np.float32(2)
    iod = np.float32(np.sqrt(np.float64(np.float32(left[0] - right[0])) ** 2 + np.float64(np.float32(left[1] - right[1])) ** 2))
    assert np.float32(float(out["iod"])) == iod
    assert out["intersect"] == "0 0 10 10"
    import oracle
    assert np.float32(float(out["area"])) == np.float32(oracle.area_under_curve(-1.0, 1.0, 0.0, 1.0))
    assert out["constants"] == "0.899999976 5 0.0500000007 0.0900000036"
    assert out["scaled"] == "4 4"  # cvRound(3.5) = 4, cvRound(4.5) = 4
    assert out["initialized"] == "0"


def _configs(reference_tree, image_dir, tmp):
    """config_*.txt of the reference tree with the image path (first value) pointing at the PPM annotation file."""
    out = []
    for key in ("hp", "ffd"):
        lines = open(reference_tree[key]).read().split("\n")
        lines[1] = str(image_dir / "index.txt")
        p = tmp / os.path.basename(str(reference_tree[key]))
        p.write_text("\n".join(lines))
        out.append(p)
    return out


def test_missing_cascade_leaves_it_uninitialized(exe, reference_tree, image_dir, tmp_path):
    """like the reference's constructor (FaceForest.cpp:23-27), a FaceForest whose cascade does not load
    (a missing file, an empty path, a file that is not a cascade) is not initialised; no GPU is reached."""
    hp, ffd = _configs(reference_tree, image_dir, tmp_path)
    env = dict(os.environ, FFD_MODEL_CACHE=str(tmp_path / "cache"))
    env.pop("FFD_MODEL", None)
    (tmp_path / "cache").mkdir()
    junk = tmp_path / "junk.xml"
    junk.write_text("<opencv_storage><nothing/></opencv_storage>")
    for cascade in (tmp_path / "missing.xml", junk):
        r = _run(exe, "init", hp, ffd, cascade, env=env)
        assert r.returncode == 0 and "initialized 0" in r.stdout, (cascade, r.stdout, r.stderr)
        assert "Error loading" in r.stderr and "cascade" in r.stderr.lower(), r.stderr
    # the bundled cascade converts (the model is built; without a device the engine itself then fails)
    r = _run(exe, "init", hp, ffd, reference_tree["xml"], env=env)
    assert r.returncode == 0 and "cascade" not in r.stderr.lower(), r.stderr


@pytest.mark.gpu
def test_eval_ffd_main(exe, reference_tree, image_dir, tmp_path, fixtures):
    from face_alignment_cvpr_2012_amd import eval as fe
    hp, ffd = _configs(reference_tree, image_dir, tmp_path)
    (tmp_path / "output").mkdir()
    env = dict(os.environ, FFD_MODEL_CACHE=str(reference_tree["cache"]))
    env.pop("FFD_MODEL", None)
    r = _run(exe, "eval", hp, ffd, reference_tree["xml"], cwd=tmp_path, env=env)
    assert r.returncode == 0, r.stderr
    g = np.load(os.path.join(GOLDEN, "oracle_golden.npz"))
    names = [str(n) for n in fixtures["names"]]
    want = [fe.landmark_errors(fixtures["parts"][names.index(u)], g["points"][names.index(u)]) for u in TEST_SPLIT]
    assert (tmp_path / "output" / "errors.txt").read_text() == fe.format_errors(want)


def truncated_cascade(xml_text, keep):
    """The cascade's first `keep` stages (a second, looser classifier of the same format)."""
    i = xml_text.index("<stages>")
    j = xml_text.index("</stages>")
    starts = [m.start() for m in re.finditer(r"<maxWeakCount>", xml_text[i:j])]
    cut = i + starts[keep]
    cut = xml_text.rindex("<_>", i, cut)
    out = xml_text[:cut] + xml_text[j:]
    return re.sub(r"<stageNum>\d+</stageNum>", "<stageNum>%d</stageNum>" % keep, out)


@pytest.mark.gpu
def test_detect_face_uses_its_classifier(exe, reference_tree, image_dir, tmp_path, fixtures, model_path):
    import face_alignment_cvpr_2012_amd as ffd
    import oracle
    second = tmp_path / "second_cascade.xml"
    second.write_text(truncated_cascade(open(reference_tree["xml"]).read(), 12))
    # the CPU restatement of the second cascade: a model converted with it (forests of the reference tree)
    model2 = ffd.convert_model(str(reference_tree["hp"]), str(reference_tree["ffd"]), str(second),
                               str(tmp_path / "model2.bin"))
    differ = 0
    try:
        for k in (0, 4, 9, 13):
            ppm = image_dir / str(fixtures["names"][k])
            got = {}
            for tag, xml, mdl in (("full", reference_tree["xml"], model_path), ("second", second, str(model2))):
                r = _run(exe, "detect", xml, ppm)
                assert r.returncode == 0, r.stdout + r.stderr
                boxes = [[int(v) for v in line.split()[1:]] for line in r.stdout.splitlines() if line.startswith("box")]
                oracle.load_model(mdl)
                want = oracle.detect_faces(fixtures["images"][k])
                assert np.array_equal(np.array(boxes, np.int32).reshape(-1, 4), want), (tag, k, boxes, want)
                got[tag] = boxes
            differ += got["full"] != got["second"]
    finally:
        oracle.load_model(model_path)
    assert differ > 0  # the looser classifier finds other boxes: the argument is the one that runs
    r = _run(exe, "detect", tmp_path / "missing.xml", image_dir / str(fixtures["names"][0]))
    assert r.returncode == 5 and "load failed" in r.stdout


@pytest.mark.gpu
def test_demo_analyze_image(exe, reference_tree, image_dir, tmp_path, fixtures, engine):
    hp, ffd = _configs(reference_tree, image_dir, tmp_path)
    env = dict(os.environ, FFD_MODEL_CACHE=str(reference_tree["cache"]))
    env.pop("FFD_MODEL", None)
    for k in (1, 7):
        r = _run(exe, "analyze", hp, ffd, reference_tree["xml"], image_dir / str(fixtures["names"][k]), env=env)
        assert r.returncode == 0, r.stderr
        faces = engine.analyzeImage(fixtures["images"][k])
        assert "orphaned_sample_fails 1" in r.stdout  # an ImageSample outliving its FaceForest
        lines = [line.split()[1:] for line in r.stdout.splitlines() if line.startswith("face")]
        assert len(lines) == len(faces) >= 1
        for v, f in zip(lines, faces):
            assert [int(x) for x in v[:4]] == list(f.bbox)
            assert np.float32(float(v[4])) == np.float32(f.headpose)
            assert np.array_equal(np.array(v[5:], np.int32).reshape(10, 2), f.ffd_cordinates)


@pytest.mark.gpu
def test_demo_train_tree(exe, image_dir, tmp_path):
    out = tmp_path / "trees"
    out.mkdir()
    r = _run(exe, "train", os.path.join(GOLDEN, "config_ffd.txt"), image_dir / "index.txt", 6, out,
             env=dict(os.environ, FFD_SPLIT_SEED="7"))
    assert r.returncode == 0, r.stdout + r.stderr
    vals = dict(zip(r.stdout.split()[0::2], r.stdout.split()[1::2]))
    assert int(vals["samples"]) == 6 * 60 and int(vals["nodes"]) > 1
    assert vals["same_archive"] == "1" and vals["saved_equal"] == "1"
