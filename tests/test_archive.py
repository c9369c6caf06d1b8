"""Boost text-archive writer (/root/reference/include/Tree.hpp:239-256 and the
serializers of App. A): the converted pretrained model re-emitted through the C ABI equals every one
of the 115 shipped tree files byte for byte (digests in tests/golden/archive_digests.json, made by
tests/golden/make_archive_digests.py from the reference's own files), and a synthetic forest survives
write -> ffd_convert -> read unchanged.  Host code only: no GPU."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from face_alignment_cvpr_2012_amd import FFDError
from face_alignment_cvpr_2012_amd import model as fmodel
from face_alignment_cvpr_2012_amd.archive import FFD, HEADPOSE, ModelArchive

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFERENCE = os.environ.get("FFD_REFERENCE", "/root/reference")
DIGESTS = json.load(open(os.path.join(REPO, "tests", "golden", "archive_digests.json")))


@pytest.fixture(scope="module")
def archive(model_path):
    with ModelArchive(model_path) as m:
        yield m


def test_tree_counts_and_save_paths(archive):
    assert archive.num_trees(HEADPOSE) == 15 and archive.num_trees(FFD) == 100
    paths = [archive.save_path(HEADPOSE, t) for t in range(15)] + [archive.save_path(FFD, t) for t in range(100)]
    assert sorted(paths) == sorted(DIGESTS)
    assert archive.save_path(FFD, 27) == "data/trees_ffd/forest_1/tree_007.txt"  # forest-major


def test_every_shipped_tree_reemitted_byte_exact(archive):
    bad = []
    for kind in (HEADPOSE, FFD):
        for t in range(archive.num_trees(kind)):
            p = archive.save_path(kind, t)
            b = archive.tree_bytes(kind, t)
            want = DIGESTS[p]
            if len(b) != want["bytes"] or hashlib.sha256(b).hexdigest() != want["sha256"]:
                bad.append(p)
    assert not bad, bad


@pytest.mark.reference
def test_save_tree_equals_reference_file(archive, tmp_path):
    if not os.path.isdir(os.path.join(REFERENCE, "data")):
        pytest.skip("reference tree not present")
    for kind, t in ((HEADPOSE, 3), (FFD, 64)):
        p = archive.save_path(kind, t)
        out = tmp_path / "tree.txt"
        archive.save_tree(kind, t, str(out))
        assert out.read_bytes() == open(os.path.join(REFERENCE, p), "rb").read(), p


def test_errors(archive, tmp_path):
    with pytest.raises(FFDError):
        archive.tree_bytes(2, 0)
    with pytest.raises(FFDError):
        archive.tree_bytes(FFD, 100)
    with pytest.raises(FFDError):
        archive.save_tree(HEADPOSE, 0, str(tmp_path / "no_such_dir" / "t.txt"))
    with pytest.raises(FFDError) as e:
        ModelArchive(str(tmp_path / "missing.bin"))
    assert "cannot open" in str(e.value)


CONFIG = """____Path to images index file
images.txt
____Path to trees
{trees}
____Number of trees
{ntrees}
____Number of tests
2500
____Max depth
{depth}
____Min patches per node
20
____Images per class
600
____Patches per image
150
____Face size
125
____Patch size ratio
0.250000
____Features
0 1 2
"""


def test_synthetic_forest_round_trip(model_path, tmp_path):
    """ffd_synth_forest (no archive-only fields: defaults) -> archives -> ffd_convert -> same arrays."""
    src = tmp_path / "synth.bin"
    subprocess.run([f"{REPO}/face_alignment_cvpr_2012_amd/bin/ffd_synth_forest", model_path, str(src), "5", "3", "9"],
                   check=True, capture_output=True)
    root = tmp_path / "root"
    with ModelArchive(str(src)) as m:
        n_hp, n_mp = m.num_trees(HEADPOSE), m.num_trees(FFD)
        for t in range(n_hp):
            d = root / m.save_path(HEADPOSE, t)
            d.parent.mkdir(parents=True, exist_ok=True)
            m.save_tree(HEADPOSE, t, str(d))
        for t in range(n_mp):
            d = root / "data" / "trees_ffd" / "forest_0" / f"tree_{t:03d}.txt"
            d.parent.mkdir(parents=True, exist_ok=True)
            m.save_tree(FFD, t, str(d))
        head = m.tree_bytes(FFD, 0)[:200].decode()
    assert head.startswith("22 serialization::archive 10 0 0 63 63 0 0 ")  # 2^5 - 1 nodes, i_node == m_num_nodes
    (root / "data" / "config_headpose.txt").write_text(CONFIG.format(trees="data/trees_headpose", ntrees=n_hp, depth=15))
    (root / "data" / "config_ffd.txt").write_text(CONFIG.format(trees="data/trees_ffd", ntrees=n_mp, depth=5))
    back = tmp_path / "back.bin"
    subprocess.run([f"{REPO}/face_alignment_cvpr_2012_amd/bin/ffd_convert", str(root), str(back)], check=True,
                   capture_output=True)
    a, b = fmodel.load(str(src)), fmodel.load(str(back))

    def as_written(x):  # Boost writes floats with 8 significant digits (digits10 + 2): lossy for some
        return np.array([float(f"{v:.8g}") for v in np.asarray(x, np.float64).ravel()], np.float32).reshape(x.shape)

    for name in ("hp.node_split", "hp.node_leaf", "hp.leaf_n", "hp.leaf_fg", "hp.leaf_labels", "hp.node_info",
                 "mp.tree_node_off", "mp.node_split", "mp.node_leaf", "mp.leaf_n", "mp.leaf_fg", "mp.leaf_offset",
                 "mp.leaf_var", "mp.leaf_pf"):
        want = as_written(a[name]) if a[name].dtype == np.float32 else a[name]
        np.testing.assert_array_equal(want, b[name], err_msg=name)
    assert not b["mp.node_info"].any()
