"""The header-only C++ drop-in (include/FaceForest.hpp) through examples/analyze_face.cpp:
the reference's analyzeFace call contract from C++ (eval_ffd.cpp:89, demo.cpp:149)."""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "examples", "build", "analyze_face")


def _run(model_path, img, box, tmp_path):
    path = tmp_path / "img.bgr"
    np.ascontiguousarray(img).tofile(path)
    h, w = img.shape[:2]
    return subprocess.run([EXE, model_path, str(path), str(w), str(h)] + [str(int(v)) for v in box],
                          capture_output=True, text=True, timeout=300)


def test_shim_reports_missing_device(model_path, fixtures, tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    assert os.path.exists(EXE), "run `make` (__graft_entry__.build())"
    r = _run(model_path, fixtures["images"][0], fixtures["boxes"][0], tmp_path)
    assert r.returncode == 3 and "no HIP device" in r.stderr


@pytest.mark.gpu
def test_shim_matches_python_engine(model_path, fixtures, engine, tmp_path):
    for i in (0, 7):
        img, box = fixtures["images"][i], tuple(int(v) for v in fixtures["boxes"][i])
        r = _run(model_path, img, box, tmp_path)
        assert r.returncode == 0, r.stderr
        vals = r.stdout.split()
        face = engine.analyzeFace(img, box)
        assert np.float32(float(vals[0])) == np.float32(face.headpose)
        assert np.array_equal(np.array(vals[1:], np.int32).reshape(10, 2), face.ffd_cordinates)
