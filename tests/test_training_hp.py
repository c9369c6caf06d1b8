"""Head-pose tree training: the HIP trainer (libffd.so ffd_train_hp_tree,
csrc/ffd_train.*: k_hp_items / k_hp_split) against the CPU restatement of train_headpose.cpp +
Tree<HeadPoseSample> (oracle/ffd_train_oracle.cpp), bit for bit: every split (channel, rectangles,
threshold), its f64 gain, the split mode drawn for it, every HeadPoseLeaf and the sampled patches.
Parity with the reference itself is unpinned (no LFW, no OpenCV / Boost, std::time(NULL) split seeds).

What the tests pin down on the restatement beyond self-consistency:
  * the split mode is the tree generator's next U{0..100} draw per SEARCHED node in depth-first order
    (Tree.hpp:267-274): the modes of the split nodes replayed from the generator after the patch draws;
  * evalSplit's two measures (HeadPoseSample.cpp:64-87,120-143,228-248) recomputed in Python for the root
    from the routed samples;
  * the patch sampling rules (positives inside the face region, background patches disjoint from the box).
"""
import functools
import math
import os

import numpy as np
import pytest

from face_alignment_cvpr_2012_amd.synthetic import headpose_training_images

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "train_hp_golden.npz")
SMALL = dict(max_depth=8, min_patches=20, ntests=50, npatches=60, tree_seed=2, split_seed=77)
N_SMALL = 10
KEYS = ("node_leaf", "node_split", "node_info", "node_mode", "leaf_n", "leaf_fg", "leaf_labels", "samples")


@functools.lru_cache(maxsize=4)
def _oracle_cached(n, items):
    import oracle
    images, faces, poses = headpose_training_images(n)
    return images, faces, poses, oracle.train_hp_tree(images, faces, poses, **dict(items))


def _oracle(n, **kw):
    return _oracle_cached(n, tuple(sorted(kw.items())))


def _children(node_leaf):
    n = len(node_leaf)
    right = np.full(n, -1)

    def walk(i):
        if node_leaf[i] >= 0:
            return i + 1
        j = walk(i + 1)
        right[i] = j
        return walk(j)
    walk(0)
    return right


def _value(I, s, x, y):
    c = I[s[0]].astype(np.int64)

    def mean(rx, ry, rw, rh):
        S = c[y + ry + rh, x + rx + rw] - c[y + ry, x + rx + rw] - c[y + ry + rh, x + rx] + c[y + ry, x + rx]
        return S // (rw * rh)
    return mean(*s[1:5]) - mean(*s[5:9])


def _mt_uniform(rng_out, lo, hi):
    """boost::uniform_int over a python iterator of mt19937 outputs (bucket division with rejection)."""
    rng = hi - lo
    if rng == 0:
        return lo
    bucket = 0xFFFFFFFF // (rng + 1)
    if 0xFFFFFFFF % (rng + 1) == rng:
        bucket += 1
    while True:
        r = next(rng_out) // bucket
        if r <= rng:
            return lo + r


class _MT:
    """std::mt19937 (== boost::mt19937), pure Python."""

    def __init__(self, seed):
        self.mt = [0] * 624
        self.mt[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            self.mt[i] = (1812433253 * (self.mt[i - 1] ^ (self.mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.i = 624

    def __iter__(self):
        return self

    def __next__(self):
        if self.i >= 624:
            for k in range(624):
                y = (self.mt[k] & 0x80000000) | (self.mt[(k + 1) % 624] & 0x7FFFFFFF)
                self.mt[k] = self.mt[(k + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            self.i = 0
        y = self.mt[self.i]
        self.i += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y


def test_hp_oracle_tree_is_consistent():
    import oracle
    images, faces, poses, a = _oracle(N_SMALL, **SMALL)
    S = a["samples"]
    ps = 31
    # sampling: 48 positives per image inside the face region, up to 12 background patches off the box
    for i in range(N_SMALL):
        pos, neg = S[(S[:, 0] == i) & (S[:, 3] >= 0)], S[(S[:, 0] == i) & (S[:, 3] < 0)]
        assert len(pos) == 48 and len(neg) <= 12 and (pos[:, 3] == poses[i] + 2).all()
        x, y, w, h = faces[i]
        assert ((pos[:, 1] >= x) & (pos[:, 1] <= x + 125 - ps - 1) & (pos[:, 2] >= y) & (pos[:, 2] <= y + 125 - ps - 1)).all()
        assert ((neg[:, 1] + ps <= x) | (neg[:, 1] >= x + w) | (neg[:, 2] + ps <= y) | (neg[:, 2] >= y + h)).all()
    assert a["i_node"] == 2 ** SMALL["max_depth"] - 1
    assert a["leaf_n"].sum() == len(S)
    split = a["node_leaf"] < 0
    assert ((a["node_mode"][split] >= 0) & (a["node_mode"][split] <= 100)).all() and (a["node_mode"][~split] == -1).all()
    # route every patch with the training rule (value < threshold -> left): leaf counts, labels, fg
    chans = [oracle.channels(im) for im in images]
    right = _children(a["node_leaf"])
    counts = np.zeros(len(a["leaf_n"]), np.int64)
    labels = np.zeros((len(a["leaf_n"]), 5), np.int64)
    for img, x, y, lab in S:
        i = 0
        while a["node_leaf"][i] < 0:
            s = a["node_split"][i]
            i = i + 1 if _value(chans[img], s, x, y) < s[9] else right[i]
        counts[a["node_leaf"][i]] += 1
        if lab >= 0:
            labels[a["node_leaf"][i], lab] += 1
    assert np.array_equal(counts, a["leaf_n"])
    assert np.array_equal(labels, a["leaf_labels"])
    np.testing.assert_array_equal(a["leaf_fg"], (labels.sum(1) / counts).astype(np.float32))


def test_hp_split_modes_follow_the_tree_generator():
    """The modes are the tree generator's U{0..100} draws after the patch draws, one per searched node in
    depth-first order (Tree.hpp:267-274), replayed here with a pure-Python mt19937."""
    images, faces, poses, a = _oracle(N_SMALL, **SMALL)
    g = _MT(SMALL["tree_seed"])
    for i in range(N_SMALL):  # replay the patch draws (train_headpose.cpp:98-134)
        for _ in range(48):
            _mt_uniform(g, 0, 125 - 31 - 1), _mt_uniform(g, 0, 125 - 31 - 1)
        H, W = images[i].shape
        x0, y0, w, h = faces[i]
        for _ in range(12):
            for attempt in range(1, 101):
                x, y = _mt_uniform(g, 0, W - 31 - 1), _mt_uniform(g, 0, H - 31 - 1)
                if x + 31 <= x0 or x >= x0 + w or y + 31 <= y0 or y >= y0 + h:
                    break
    # pre-order: a node draws a mode when it is searched (>= min_patches samples above max_depth), whether
    # or not a split is found; leaves record -1, split nodes the mode they drew
    depth, stack = [], [0]
    for v in a["node_leaf"]:
        d = stack.pop()
        depth.append(d)
        if v < 0:
            stack += [d + 1, d + 1]
    modes, expect = [], []
    for v, m, d in zip(a["node_leaf"], a["node_mode"], depth):
        if v < 0:
            modes.append(int(m))
            expect.append(_mt_uniform(g, 0, 100))
        elif a["leaf_n"][v] >= SMALL["min_patches"] and d < SMALL["max_depth"]:
            _mt_uniform(g, 0, 100)  # searched, no valid split
    assert modes == expect


def test_hp_root_gain_recomputed():
    """evalSplit of the root's chosen split recomputed from the routed patches in Python (entropie or
    gain2 by the root's mode; math.log vs the restated log: 1e-12 relative)."""
    import oracle
    images, faces, poses, a = _oracle(N_SMALL, **SMALL)
    chans = [oracle.channels(im) for im in images]
    s = a["node_split"][0]
    left = np.array([_value(chans[img], s, x, y) < s[9] for img, x, y, _ in a["samples"]])
    lab = a["samples"][:, 3]

    def entropie(L):
        n, p = len(L), float((L >= 0).sum())
        e = 0.0
        for q in (p / n, (n - p) / n):
            if q > 0:
                e += q * math.log(q)
        return e

    def gain2(L):
        P = L[L >= 0].astype(np.float64)
        m = P.sum() / len(P)
        return -((P * P).sum() / len(P) - m * m), len(P)
    A, B = lab[left], lab[~left]
    if a["node_mode"][0] < 50:
        want = (entropie(A) * len(A) + entropie(B) * len(B)) / len(lab)
    else:
        (ga, na), (gb, nb) = gain2(A), gain2(B)
        want = (ga * na + gb * nb) / (na + nb)
    assert abs(a["node_info"][0] - want) <= 1e-12 * abs(want)


def test_hp_oracle_matches_committed_golden():
    g = np.load(GOLDEN, allow_pickle=False)
    kw = {k: int(g["param"][i]) for i, k in enumerate(("max_depth", "min_patches", "ntests", "npatches", "tree_seed",
                                                        "split_seed"))}
    _, _, _, a = _oracle(int(g["n_images"]), **kw)
    for k in KEYS:
        assert np.array_equal(a[k], g[k]), k
    assert a["i_node"] == int(g["i_node"])


def _gpu_tree(n, archive_path=None, **kw):
    from face_alignment_cvpr_2012_amd.training import ForestParam, train_hp_tree
    images, faces, poses = headpose_training_images(n)
    p = ForestParam.headpose(max_depth=kw["max_depth"], min_patches=kw["min_patches"], ntests=kw["ntests"],
                             npatches=kw["npatches"])
    return train_hp_tree(images, faces, poses, p, tree_seed=kw["tree_seed"], split_seed=kw["split_seed"])


@pytest.mark.gpu
def test_gpu_hp_training_matches_oracle_small():
    _, _, _, a = _oracle(N_SMALL, **SMALL)
    t = _gpu_tree(N_SMALL, **SMALL)
    assert t.kind == 0
    b = t.arrays()
    for k in KEYS:
        assert np.array_equal(a[k], b[k]), k
    st = t.stats
    assert st["samples"] == len(a["samples"]) and st["items"] == SMALL["ntests"] * int((a["node_leaf"] < 0).sum())


@pytest.mark.gpu
def test_gpu_hp_training_matches_golden(tmp_path):
    from test_model import _parse_archive
    g = np.load(GOLDEN, allow_pickle=False)
    md, mp_, nt, npch, ts, ss = (int(v) for v in g["param"])
    t = _gpu_tree(int(g["n_images"]), max_depth=md, min_patches=mp_, ntests=nt, npatches=npch, tree_seed=ts,
                  split_seed=ss)
    b = t.arrays()
    for k in KEYS:
        assert np.array_equal(g[k], b[k]), k
    path = tmp_path / "tree_000.txt"
    t.save(str(path))
    data = path.read_bytes()
    assert data == t.archive()
    assert data.startswith(b"22 serialization::archive 10 0 0 %d %d " % (2 ** md - 1, int(g["i_node"])))
    infos = []
    finished, splits, leaves = _parse_archive(str(path), True, infos)
    assert finished
    assert np.array_equal(np.array(splits, np.int16), g["node_split"][g["node_leaf"] < 0])
    assert [x[0] for x in leaves] == list(g["leaf_n"])
    assert np.array_equal(np.array([x[2] for x in leaves], np.int32), g["leaf_labels"])
    assert [float(x) for x in infos] == list(g["node_info"][g["node_leaf"] < 0])


@pytest.mark.gpu
def test_gpu_hp_training_rejects_bad_input():
    from face_alignment_cvpr_2012_amd import FFDError
    from face_alignment_cvpr_2012_amd.training import ForestParam, train_hp_tree
    images, faces, poses = headpose_training_images(2)
    p = ForestParam.headpose(ntests=4, npatches=10)
    with pytest.raises(FFDError):  # face box leaves no room for the positive patches
        train_hp_tree(images, faces + np.array([100, 0, 0, 0]), poses, p)
    with pytest.raises(FFDError):
        train_hp_tree(images, faces, np.array([3, 0]), p)
    with pytest.raises(ValueError):
        train_hp_tree(images, faces[:1], poses, p)
