import gzip
import os
import shutil
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

MODEL = os.path.join(REPO, "model", "ffd_model.bin")
REFERENCE = os.environ.get("FFD_REFERENCE", "/root/reference")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "reference: needs the read-only reference tree at /root/reference")


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first():
    """PyTorch's HIP runtime first: a test that creates an engine before any torch.cuda call would
    otherwise leave torch without devices for the tests that hand it torch buffers."""
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()


@pytest.fixture(scope="session")
def model_path():
    if not os.path.exists(MODEL):
        pytest.fail(f"model not converted: {MODEL} (run __graft_entry__.build())")
    return MODEL


@pytest.fixture(scope="session")
def fixtures():
    from face_alignment_cvpr_2012_amd.synthetic import load_fixtures
    return load_fixtures()


@pytest.fixture(scope="session")
def oracle_mod(model_path):
    import oracle
    oracle.load_model(model_path)
    return oracle


@pytest.fixture(scope="session")
def engine(model_path):
    import face_alignment_cvpr_2012_amd as ffd
    import torch
    if torch.cuda.is_available():  # PyTorch's HIP runtime first: tests hand torch buffers to the engine
        torch.cuda.init()
    ff = ffd.FaceForest(ffd.FaceForestOptions(model_path=model_path))
    yield ff
    ff.close()


@pytest.fixture(scope="session")
def reference_root():
    if not os.path.isdir(os.path.join(REFERENCE, "data")):
        pytest.skip("reference tree not present (only in the build container)")
    return REFERENCE


def crops(n, seed=2012):
    from face_alignment_cvpr_2012_amd.synthetic import make_crops
    return make_crops(n, seed=seed)[0]


@pytest.fixture(scope="session")
def reference_tree(tmp_path_factory, model_path):
    """data/trees_headpose + data/trees_ffd/forest_{0..4} archives, the two configs pointing at them, the cascade."""
    from face_alignment_cvpr_2012_amd import archive
    root = tmp_path_factory.mktemp("reference_data")
    with archive.ModelArchive(model_path) as m:
        m.save_all(str(root))
    cfg = {}
    for name, sub in (("config_headpose.txt", "data/trees_headpose"), ("config_ffd.txt", "data/trees_ffd")):
        lines = open(os.path.join(os.path.join(REPO, "tests", "golden"), name)).read().split("\n")
        lines[3] = str(root / sub)  # the "Path to trees" value (loadConfigFile's second pair)
        cfg[name] = root / name
        cfg[name].write_text("\n".join(lines))
    xml = root / "haarcascade_frontalface_alt.xml"
    with gzip.open(os.path.join(os.path.join(REPO, "tests", "golden"), "haarcascade_frontalface_alt.xml.gz")) as src, open(xml, "wb") as dst:
        shutil.copyfileobj(src, dst)
    cache = root / "cache"
    cache.mkdir()
    return {"root": root, "hp": cfg["config_headpose.txt"], "ffd": cfg["config_ffd.txt"], "xml": xml, "cache": cache}
