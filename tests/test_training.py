"""Facial-feature tree training: the HIP trainer (libffd.so ffd_train_mp_tree,
csrc/ffd_train.*) against the CPU restatement (oracle/ffd_train_oracle.cpp), bit for bit: every split
(channel, rectangles, threshold), every split's information gain (f64), every MPLeaf payload and the
sampled patches.  Parity with the reference itself is unpinned: it needs OpenCV 2.4.9, Boost 1.55 and the
LFW training set, and seeds its split generators with std::time(NULL) (SplitGen.hpp:78).

Reference behaviour the tests pin down on the restatement:
  * applyOptimalSplit sends value < threshold to the left child (lower_bound, SplitGen.hpp:113) while
    inference goes left on value <= threshold (MPSample::eval, MPSample.cpp:77-84): routing the training
    samples with the TRAINING rule reproduces every leaf's sample count;
  * a finished tree has i_node == m_num_nodes == 2^max_depth - 1 (Tree.hpp:53,72-79,110,139).
"""
import math
import os
import struct

import numpy as np
import pytest

from face_alignment_cvpr_2012_amd.synthetic import training_rois

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "train_golden.npz")
SMALL = dict(max_depth=8, min_patches=20, ntests=60, npatches=40, tree_seed=3, split_seed=2012)


def _oracle_tree(n_img, **kw):
    import oracle
    rois, parts = training_rois(n_img)
    return rois, parts, oracle.train_mp_tree(rois, parts, **kw)


def _ulp(x):
    return math.ulp(x)


def test_log_within_one_ulp():
    import oracle
    rng = np.random.default_rng(5)
    xs = np.concatenate([rng.uniform(0, 1, 3000), np.exp(rng.uniform(-700, 700, 3000)), [1.0, 0.5, 2.0, 1e-310, 5e-324],
                         np.nextafter(1.0, 0) - rng.uniform(0, 1e-9, 200), 1 + rng.uniform(0, 1e-9, 200)])
    for x in xs:
        if x <= 0:
            continue
        got, want = oracle.log(float(x)), math.log(float(x))
        assert abs(got - want) <= _ulp(want) or got == want, (x, got, want)


def _route(rois, parts_unused, a, ps=31):
    """Send every training sample down the tree with the training rule (value < thr -> left)."""
    import oracle
    chans = [oracle.channels(r) for r in rois]  # [38][h+1][w+1] u32
    leaf_of_node = a["node_leaf"]
    # pre-order children: left = i + 1, right = after the left subtree
    n = len(leaf_of_node)
    right = np.full(n, -1)

    def walk(i):
        if leaf_of_node[i] >= 0:
            return i + 1
        j = walk(i + 1)
        right[i] = j
        return walk(j)
    walk(0)
    counts = np.zeros(len(a["leaf_n"]), np.int64)
    for img, x, y in a["samples"]:
        I = chans[img].astype(np.int64)
        i = 0
        while leaf_of_node[i] < 0:
            s = a["node_split"][i]

            def mean(rx, ry, rw, rh):
                c = I[s[0]]
                S = c[y + ry + rh, x + rx + rw] - c[y + ry, x + rx + rw] - c[y + ry + rh, x + rx] + c[y + ry, x + rx]
                return S // (rw * rh)
            v = mean(*s[1:5]) - mean(*s[5:9])
            i = i + 1 if v < s[9] else right[i]
        counts[leaf_of_node[i]] += 1
    return counts


def test_oracle_tree_is_consistent():
    rois, parts, a = _oracle_tree(20, **SMALL)
    assert a["i_node"] == 2 ** SMALL["max_depth"] - 1
    assert a["leaf_n"].sum() == 20 * SMALL["npatches"]
    assert (a["leaf_n"] >= 2).all()
    assert np.array_equal(_route(rois, parts, a), a["leaf_n"])
    split = a["node_leaf"] < 0
    assert split.sum() + len(a["leaf_n"]) == len(a["node_leaf"])
    assert (a["node_info"][split] < 0).all() and (a["node_info"][~split] == 0).all()  # sum p log p < 0
    s = a["node_split"][split]
    assert ((s[:, 0] >= 0) & (s[:, 0] < 38)).all()
    assert ((s[:, [3, 4, 7, 8]] >= 1) & (s[:, [3, 4, 7, 8]] <= 22)).all()
    assert ((s[:, 1] + s[:, 3] < 31) & (s[:, 6] + s[:, 8] < 31)).all()
    # leaf payloads: the fg fraction and the sample count agree; pf in [0, 1]
    assert ((a["leaf_fg"] >= 0) & (a["leaf_fg"] <= 1)).all() and ((a["leaf_pf"] >= 0) & (a["leaf_pf"] <= 1)).all()


def test_oracle_matches_committed_golden():
    """The committed golden (tests/golden/make_train_golden.py) is reproduced by the restatement."""
    g = np.load(GOLDEN, allow_pickle=False)
    kw = {k: int(g["param"][i]) for i, k in enumerate(("max_depth", "min_patches", "ntests", "npatches", "tree_seed",
                                                        "split_seed"))}
    _, _, a = _oracle_tree(int(g["n_images"]), **kw)
    for k in ("node_leaf", "node_split", "node_info", "leaf_n", "leaf_fg", "leaf_offset", "leaf_var", "leaf_pf", "samples"):
        assert np.array_equal(a[k], g[k]), k


@pytest.mark.gpu
def test_gpu_training_matches_oracle_small():
    from face_alignment_cvpr_2012_amd.training import ForestParam, train_mp_tree
    rois, parts, a = _oracle_tree(20, **SMALL)
    p = ForestParam(max_depth=SMALL["max_depth"], min_patches=SMALL["min_patches"], ntests=SMALL["ntests"],
                    npatches=SMALL["npatches"])
    t = train_mp_tree(rois, parts, p, tree_seed=SMALL["tree_seed"], split_seed=SMALL["split_seed"])
    b = t.arrays(n_samples=20 * SMALL["npatches"])
    for k in ("samples", "node_leaf", "node_split", "node_info", "leaf_n", "leaf_fg", "leaf_offset", "leaf_var", "leaf_pf"):
        assert np.array_equal(a[k], b[k]), k
    st = t.stats
    assert st["samples"] == 20 * SMALL["npatches"] and st["levels"] >= 2


@pytest.mark.gpu
def test_gpu_training_matches_oracle_large_patch():
    """A 60 x 60 patch (face_size 240 x patch_size_ratio 0.25; the trainer accepts up to 64): rectangles up to
    47 x 47 (area 2,209), past the 484 up to which the fused rcp quotient is proven; those take the integer
    quotient (ffd_train.hip eval_sample), equal to (int)(S / (float)area) there."""
    from face_alignment_cvpr_2012_amd.training import ForestParam, train_mp_tree
    kw = dict(SMALL, max_depth=6)
    rois, parts = training_rois(8, face_size=240)
    a = __import__("oracle").train_mp_tree(rois, parts, face_size=240, **kw)
    p = ForestParam(max_depth=kw["max_depth"], min_patches=kw["min_patches"], ntests=kw["ntests"],
                    npatches=kw["npatches"], face_size=240)
    assert p.getPatchSize() == 60
    t = train_mp_tree(rois, parts, p, tree_seed=kw["tree_seed"], split_seed=kw["split_seed"])
    b = t.arrays(samples=True)
    for k in ("samples", "node_leaf", "node_split", "node_info", "leaf_n", "leaf_fg", "leaf_offset", "leaf_var", "leaf_pf"):
        assert np.array_equal(a[k], b[k]), k
    s = a["node_split"][a["node_leaf"] < 0]
    assert (s[:, 3] * s[:, 4] > 484).any() or (s[:, 7] * s[:, 8] > 484).any()  # the integer quotient ran


@pytest.mark.gpu
def test_gpu_training_matches_golden_full_config(tmp_path):
    """The reference's config_ffd.txt shape (max_depth 20, min_patches 20, 25 thresholds, patch 31 of a
    125 face) at a reduced stripe count, against the committed oracle golden; the archive parses back
    to the same splits and leaves."""
    from face_alignment_cvpr_2012_amd.training import ForestParam, train_mp_tree
    from test_model import _parse_archive
    g = np.load(GOLDEN, allow_pickle=False)
    md, mp_, nt, npch, ts, ss = (int(v) for v in g["param"])
    rois, parts = training_rois(int(g["n_images"]))
    t = train_mp_tree(rois, parts, ForestParam(max_depth=md, min_patches=mp_, ntests=nt, npatches=npch),
                      tree_seed=ts, split_seed=ss, save_path="data/trees_ffd/forest_0/tree_000.txt")
    b = t.arrays(n_samples=len(g["samples"]))
    for k in ("samples", "node_leaf", "node_split", "node_info", "leaf_n", "leaf_fg", "leaf_offset", "leaf_var", "leaf_pf"):
        assert np.array_equal(g[k], b[k]), k
    path = tmp_path / "tree_000.txt"
    t.save(str(path))
    data = path.read_bytes()
    assert data == t.archive()
    assert data.startswith(b"22 serialization::archive 10 0 0 %d %d " % (2 ** md - 1, 2 ** md - 1))
    finished, splits, leaves = _parse_archive(str(path), False)
    assert finished
    assert np.array_equal(np.array(splits, np.int16), g["node_split"][g["node_leaf"] < 0])
    assert [x[0] for x in leaves] == list(g["leaf_n"])
    assert np.array_equal(np.array([x[2] for x in leaves]).reshape(-1, 10, 2), g["leaf_offset"])

    def as_written(x):  # Boost writes floats with digits10 + 2 = 8 significant digits
        return np.array([float(f"{v:.8g}") for v in np.asarray(x, np.float64).ravel()], np.float32).reshape(x.shape)
    assert np.array_equal(np.array([x[3] for x in leaves], np.float32), as_written(g["leaf_var"]))
    assert np.array_equal(np.array([x[4] for x in leaves], np.float32), as_written(g["leaf_pf"]))
    infos = []
    _parse_archive(str(path), False, infos)
    assert [float(x) for x in infos] == list(g["node_info"][g["node_leaf"] < 0])  # %.17g round-trips f64


@pytest.mark.gpu
def test_gpu_training_rejects_bad_input():
    from face_alignment_cvpr_2012_amd import FFDError
    from face_alignment_cvpr_2012_amd.training import ForestParam, train_mp_tree
    rois, parts = training_rois(2)
    with pytest.raises(FFDError):
        train_mp_tree([rois[0][:20, :20]], parts[:1], ForestParam(ntests=4, npatches=4))
    with pytest.raises(ValueError):
        train_mp_tree(rois, parts[:1], ForestParam(ntests=4, npatches=4))


def test_training_struct_layout():
    from face_alignment_cvpr_2012_amd.training import _TrainImage, _TrainParam, _TrainStats
    import ctypes
    assert ctypes.sizeof(_TrainParam) == 8 * 4 + 3 * 8 + 4 * 4  # 7 i32 + f32, 3 pointers, 2 u32 + i32 (+ pad)
    assert ctypes.sizeof(_TrainImage) == 8 + 3 * 4 + 4 + 8
    assert ctypes.sizeof(_TrainStats) == 5 * 8 + 2 * 8 + 8
    assert struct.calcsize("d") == 8
