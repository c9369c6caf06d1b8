"""C-ABI boundary checks that need no GPU: the shared library loads, exports every entry point
include/ffd.h declares, the ctypes record layout matches the header, and the product refuses to
run without a HIP device (no CPU fallback)."""
import ctypes
import os
import re

import pytest

import face_alignment_cvpr_2012_amd as ffd

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    text = open(os.path.join(REPO, "include", "ffd.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ffd_[a-z_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(ffd.library_path())
    names = declared_functions()
    assert len(names) >= 16, names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(ffd.EXPORTED_SYMBOLS)


def test_version_and_stage_names():
    lib = ffd.lib()
    assert lib.ffd_version().decode().startswith("ffd")
    names = [lib.ffd_stage_name(i).decode() for i in range(ffd.NUM_STAGES)]
    assert names[0] == "gray_resize" and names[-1] == "meanshift" and len(set(names)) == ffd.NUM_STAGES
    assert lib.ffd_stage_name(ffd.NUM_STAGES).decode() == ""


def test_face_record_layout():
    # ffd_face: headpose, pose_variance, bbox(4 x i32), points[10][2] i32, n_trees, status
    assert ffd.FACE_RECORD_BYTES == 4 + 4 + 16 + 80 + 4 + 4 == 112


def test_no_cpu_fallback_without_device(model_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present; covered by the gpu tests")
    with pytest.raises(ffd.FFDError) as e:
        ffd.FaceForest(ffd.FaceForestOptions(model_path=model_path))
    assert "no HIP device" in str(e.value)
