"""Model converter pinned against the reference's own tree archives.

Known-answer values were computed from /root/reference/data/trees_*;
the converter (csrc/ffd_convert.cpp) must reproduce them exactly.  The `reference`-marked test
re-parses one archive with an independent pure-Python reader (build container only).
"""
import os

import numpy as np
import pytest

from face_alignment_cvpr_2012_amd import model as fm

# forest: (trees, total nodes, leaves, (tree_000 nodes, leaves, sum thr), (last tree nodes, leaves, sum thr))
KAT = {
    "hp": (15, 176841, 88428, (11701, 5851, 1398), (13541, 6771, 3914)),
    0: (20, 305702, 152861, (15077, 7539, 4277), (15475, 7738, 3558)),
    1: (20, 308648, 154334, (15611, 7806, 4241), (15209, 7605, 3804)),
    2: (20, 311500, 155760, (15595, 7798, 2653), (15663, 7832, 3247)),
    3: (20, 311756, 155888, (15507, 7754, 3820), (15715, 7858, 3400)),
    4: (20, 299046, 149533, (15501, 7751, 4587), (14665, 7333, 2604)),
}


@pytest.fixture(scope="module")
def m(model_path):
    return fm.load(model_path)


def test_params(m):
    hp, mp = m["hp.param"], m["mp.param"]
    # max_depth, min_patches, ntests, ntrees, nimages, npatches, face_size, n_forests
    assert list(hp) == [15, 20, 2000, 15, 400, 200, 125, 1]
    assert list(mp) == [20, 20, 2500, 20, 600, 150, 125, 5]
    assert m["hp.patch_ratio"][0] == np.float32(0.25)
    assert list(m["hp.features"]) == [0, 1, 2] and list(m["mp.features"]) == [0, 1, 2]


def test_headpose_forest_kat(m):
    trees, nodes, leaves, first, last = KAT["hp"]
    off = m["hp.tree_node_off"]
    assert len(off) - 1 == trees and off[-1] == nodes
    assert m["hp.leaf_n"].size == leaves
    assert fm.tree_stats(m, "hp", 0) == first
    assert fm.tree_stats(m, "hp", trees - 1) == last


@pytest.mark.parametrize("forest", [0, 1, 2, 3, 4])
def test_ffd_forest_kat(m, forest):
    trees, nodes, leaves, first, last = KAT[forest]
    off = m["mp.tree_node_off"]
    lo, hi = forest * 20, forest * 20 + trees
    assert off[hi] - off[lo] == nodes
    lo_leaf = m["mp.tree_leaf_off"]
    assert lo_leaf[hi] - lo_leaf[lo] == leaves
    assert fm.tree_stats(m, "mp", lo) == first
    assert fm.tree_stats(m, "mp", hi - 1) == last


def test_structure_invariants(m):
    for p in ("hp", "mp"):
        leaf = m[p + ".node_leaf"]
        internal = leaf < 0
        sp = m[p + ".node_split"]
        # every tree is a full binary tree: leaves = internal + 1 per tree
        off = m[p + ".tree_node_off"]
        for t in range(len(off) - 1):
            b, e = off[t], off[t + 1]
            assert (leaf[b:e] >= 0).sum() == (leaf[b:e] < 0).sum() + 1
        # leaf ordinals are 0..L-1 in file order
        lv = leaf[~internal]
        assert np.array_equal(lv, np.arange(lv.size))
        s = sp[internal]
        assert s[:, 0].min() >= 0 and s[:, 0].max() <= 37
        assert s[:, [3, 4, 7, 8]].min() >= 1 and s[:, [3, 4, 7, 8]].max() <= 22
        assert (s[:, 1] + s[:, 3]).max() <= 30 and (s[:, 2] + s[:, 4]).max() <= 30
        assert s[:, 9].min() >= -256 and s[:, 9].max() <= 256
    assert m["hp.leaf_n"].min() == 2 and m["hp.leaf_n"].max() == 16714
    assert m["mp.leaf_n"].min() == 2 and m["mp.leaf_n"].max() == 918
    off = m["mp.leaf_offset"]
    assert off.shape[1:] == (10, 2)
    assert off[..., 0].min() == -110 and off[..., 0].max() == 104
    assert off[..., 1].min() == -92 and off[..., 1].max() == 142


def _parse_archive(path, hp, infos=None):
    """Independent minimal reader of one Boost text archive (grammar: SURVEY.md App. A); infos, if a
    list, receives every split's archived ThresholdSplit::info token in pre-order."""
    toks = open(path).read().split()
    it = iter(toks)
    nx = lambda: next(it)  # noqa: E731
    assert nx() == "22" and nx() == "serialization::archive" and nx() == "10"
    [nx() for _ in range(2)]
    num_nodes, i_node = int(nx()), int(nx())
    [nx() for _ in range(2 + 8)]
    for _ in range(2):
        n = int(nx())
        if n:
            nx()
    nf = int(nx()); nx(); [nx() for _ in range(nf)]  # noqa: E702
    n = int(nx())
    if n:
        nx()
    assert nx() == "3" and nx() == "1" and nx() == "0"
    splits, leaves = [], []
    first = {"leaf": True, "split": True, "vp": True}

    def node():
        nx(); nx()
        is_leaf, has_split = int(nx()), int(nx())
        if is_leaf:
            if first["leaf"]:
                nx(); nx(); first["leaf"] = False  # noqa: E702
            if hp:
                n_, fg = int(nx()), np.float32(nx())
                nx(); nx()
                leaves.append((n_, fg, [int(nx()) for _ in range(5)]))
            else:
                n_ = int(nx())
                if first["vp"]:
                    nx(); nx()  # noqa: E702
                nx(); nx()
                if first["vp"]:
                    nx(); nx(); first["vp"] = False  # noqa: E702
                pts = [int(nx()) for _ in range(20)]
                nx(); nx(); var = [np.float32(nx()) for _ in range(10)]  # noqa: E702
                nx(); nx(); pf = [np.float32(nx()) for _ in range(10)]  # noqa: E702
                leaves.append((n_, np.float32(nx()), pts, var, pf))
        if has_split:
            if first["split"]:
                [nx() for _ in range(4)]
            ch = int(nx())
            if first["split"]:
                nx(); nx(); first["split"] = False  # noqa: E702
            r = [int(nx()) for _ in range(8)]
            info = nx()
            if infos is not None:
                infos.append(info)
            splits.append([ch] + r + [int(nx())])
        if not is_leaf:
            assert nx() == "3"
            node()
            assert nx() == "3"
            node()

    node()
    return num_nodes == i_node, splits, leaves


@pytest.mark.reference
@pytest.mark.parametrize("kind,path,prefix,tree", [
    ("hp", "data/trees_headpose/tree_003.txt", "hp", 3),
    ("mp", "data/trees_ffd/forest_2/tree_011.txt", "mp", 2 * 20 + 11),
])
def test_independent_parse_matches_model(m, reference_root, kind, path, prefix, tree):
    finished, splits, leaves = _parse_archive(os.path.join(reference_root, path), kind == "hp")
    assert finished
    b, e = m[prefix + ".tree_node_off"][tree], m[prefix + ".tree_node_off"][tree + 1]
    leaf = m[prefix + ".node_leaf"][b:e]
    sp = m[prefix + ".node_split"][b:e][leaf < 0]
    assert np.array_equal(sp, np.array(splits, np.int16))
    l0, l1 = m[prefix + ".tree_leaf_off"][tree], m[prefix + ".tree_leaf_off"][tree + 1]
    assert l1 - l0 == len(leaves)
    if kind == "hp":
        assert np.array_equal(m["hp.leaf_n"][l0:l1], [x[0] for x in leaves])
        assert np.array_equal(m["hp.leaf_fg"][l0:l1], np.array([x[1] for x in leaves], np.float32))
        assert np.array_equal(m["hp.leaf_labels"][l0:l1], [x[2] for x in leaves])
    else:
        assert np.array_equal(m["mp.leaf_n"][l0:l1], [x[0] for x in leaves])
        assert np.array_equal(m["mp.leaf_fg"][l0:l1], np.array([x[1] for x in leaves], np.float32))
        assert np.array_equal(m["mp.leaf_offset"][l0:l1].reshape(-1, 20), [x[2] for x in leaves])
        assert np.array_equal(m["mp.leaf_var"][l0:l1], np.array([x[3] for x in leaves], np.float32))
        assert np.array_equal(m["mp.leaf_pf"][l0:l1], np.array([x[4] for x in leaves], np.float32))
