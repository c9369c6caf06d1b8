"""A reference main's FaceForest setup through the C++ drop-in header (examples/reference_main.cpp): eval_ffd's
loadConfigFile / FaceForestOptions{hp_forest_param, mp_forest_param, fd_option.path_face_cascade} /
FaceForest(ff_options) (src/eval_ffd.cpp:137-174) with the reference's tree directories, converted in-process by
ffd_model_convert (FaceForest.cpp:15-58, Forest.hpp:103-153) into a cached model.

Fixtures: the tree directories are the pretrained trees re-emitted as the reference's Boost archives by the
archive writer (byte-identical to the shipped files, tests/test_archive.py); the configs and the cascade are
copies of the reference's data files (tests/golden/config_*.txt, haarcascade_frontalface_alt.xml.gz)."""
import gzip
import os
import shutil
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
EXE = os.path.join(REPO, "examples", "build", "reference_main")


def _run(ref, img, box, tmp_path):
    path = tmp_path / "img.bgr"
    np.ascontiguousarray(img).tofile(path)
    h, w = img.shape[:2]
    env = dict(os.environ, FFD_MODEL_CACHE=str(ref["cache"]))
    env.pop("FFD_MODEL", None)
    return subprocess.run([EXE, str(ref["hp"]), str(ref["ffd"]), str(ref["xml"]), str(path), str(w), str(h)] +
                          [str(int(v)) for v in box], capture_output=True, text=True, timeout=600, env=env)


def test_reference_options_convert_the_tree_directories(reference_tree, fixtures, model_path, tmp_path):
    """The archives named by the options become a model whose forests and cascade equal the committed model's
    (no device needed for the conversion; without one the engine then reports it)."""
    import torch

    from face_alignment_cvpr_2012_amd import model as fm
    assert os.path.exists(EXE), "run `make` (__graft_entry__.build())"
    r = _run(reference_tree, fixtures["images"][0], fixtures["boxes"][0], tmp_path)
    if not torch.cuda.is_available():
        assert r.returncode == 3 and "no HIP device" in r.stderr, r.stderr
    else:
        assert r.returncode == 0, r.stderr
    made = [p for p in os.listdir(reference_tree["cache"]) if p.endswith(".bin")]
    assert len(made) == 1
    got, want = fm.load(str(reference_tree["cache"] / made[0])), fm.load(model_path)
    for k, v in want.items():  # (the archives carry their own tree_path strings: re-emitted byte for byte)
        assert k in got, k
        assert got[k].dtype == v.dtype and np.array_equal(got[k], v), k


@pytest.mark.gpu
def test_reference_main_matches_engine(reference_tree, fixtures, engine, tmp_path):
    for i in (0, 9):
        img, box = fixtures["images"][i], tuple(int(v) for v in fixtures["boxes"][i])
        r = _run(reference_tree, img, box, tmp_path)
        assert r.returncode == 0, r.stderr
        lines = r.stdout.splitlines()
        vals = lines[0].split()
        face = engine.analyzeFace(img, box)
        assert np.float32(float(vals[0])) == np.float32(face.headpose)
        assert np.array_equal(np.array(vals[1:], np.int32).reshape(10, 2), face.ffd_cordinates)
        assert int(lines[1]) == len(engine.detectFace(img))
