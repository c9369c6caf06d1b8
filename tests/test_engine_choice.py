"""No silent engine choice in the C++ drop-in (VERDICT r5 "next" #6): the reference's ImageSample, MeanShift::shift /
mode and Forest<S>::load carry no engine (src/ImageSample.cpp:11-20, include/MeanShift.hpp:41-76,
include/Forest.hpp:103-129).  tests/cxx/engine_choice.cpp checks that with one FaceForest alive they use its engine,
and that with two alive an engine-less call fails with an "ambiguous" error instead of binding to the
last-constructed FaceForest (CPU: the header's registry with two placeholder engines; GPU: two real FaceForests on
device 0, named engines giving the same MeanShift mode)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "cxx", "engine_choice.cpp")
LIB = os.path.join(REPO, "face_alignment_cvpr_2012_amd", "lib")


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    if not os.path.exists(os.path.join(LIB, "libffd.so")):
        pytest.skip("libffd.so not built (make)")
    out = str(tmp_path_factory.mktemp("ec") / "engine_choice")
    r = subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Werror", "-I" + os.path.join(REPO, "include"), SRC, "-o",
                        out, "-L" + LIB, "-lffd", "-Wl,-rpath," + LIB], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


def test_two_forests_make_engineless_calls_fail_cpu(exe):
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "failures 0" in r.stdout
    assert "2 FaceForests hold the trees" in r.stderr  # Forest::load refused with both alive


@pytest.mark.gpu
def test_two_forests_make_engineless_calls_fail_gpu(exe, model_path):
    r = subprocess.run([exe, "gpu", model_path], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "failures 0" in r.stdout
