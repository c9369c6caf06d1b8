"""Tree training on the GPU over the C ABI ffd_train_* (include/ffd.h): facial-feature
trees (Tree<MPSample>, train_mp_tree) and head-pose trees (Tree<HeadPoseSample>, train_hp_tree).

Mirrors the reference's training entry points: ForestParam (include/Constants.hpp:24-60, the
config_ffd.txt values by default) and trainTree (src/train_ffd.cpp:34-123) from the training ROIs on,
which grows a Tree<MPSample> (include/Tree.hpp:43-171) and saves it as the reference's Boost text
archive (Tree<S>::save, Tree.hpp:239-256).  The split search runs in libffd.so's HIP kernels; there is
no CPU fallback (the CPU restatement in oracle/ is test infrastructure).

    rois, parts = synthetic.training_rois(40)
    tree = train_mp_tree(rois, parts, ForestParam(ntests=500), tree_seed=1, split_seed=2012)
    tree.save("tree_000.txt")

    images, boxes, poses = synthetic.headpose_training_images(40)
    hp = train_hp_tree(images, boxes, poses, ForestParam.headpose(ntests=500), tree_seed=1, split_seed=2012)
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import FFDError, lib


class _TrainParam(ctypes.Structure):
    _fields_ = [("max_depth", ctypes.c_int32), ("min_patches", ctypes.c_int32), ("ntests", ctypes.c_int32),
                ("ntrees", ctypes.c_int32), ("nimages", ctypes.c_int32), ("npatches", ctypes.c_int32),
                ("face_size", ctypes.c_int32), ("patch_size_ratio", ctypes.c_float),
                ("tree_path", ctypes.c_char_p), ("image_path", ctypes.c_char_p), ("save_path", ctypes.c_char_p),
                ("tree_seed", ctypes.c_uint32), ("split_seed", ctypes.c_uint32), ("device", ctypes.c_int32)]


class _TrainImage(ctypes.Structure):
    _fields_ = [("gray", ctypes.c_void_p), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("stride", ctypes.c_int32), ("parts", ctypes.c_void_p)]


class _Rect(ctypes.Structure):
    _fields_ = [("x", ctypes.c_int32), ("y", ctypes.c_int32), ("width", ctypes.c_int32), ("height", ctypes.c_int32)]


class _TrainHpImage(ctypes.Structure):
    _fields_ = [("gray", ctypes.c_void_p), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("stride", ctypes.c_int32), ("face", _Rect), ("pose", ctypes.c_int32)]


class _TrainStats(ctypes.Structure):
    _fields_ = [("channels_ms", ctypes.c_double), ("search_ms", ctypes.c_double), ("partition_ms", ctypes.c_double),
                ("leaves_ms", ctypes.c_double), ("total_ms", ctypes.c_double), ("samples", ctypes.c_int64),
                ("items", ctypes.c_int64), ("levels", ctypes.c_int32)]


_bound = False


def _lib():
    global _bound
    L = lib()
    if not _bound:
        P = ctypes.POINTER
        L.ffd_train_param_init.argtypes = [P(_TrainParam)]
        L.ffd_train_mp_tree.argtypes = [P(_TrainParam), P(_TrainImage), ctypes.c_int32, P(ctypes.c_void_p)]
        L.ffd_train_mp_tree.restype = ctypes.c_int
        L.ffd_train_last_error.restype = ctypes.c_char_p
        L.ffd_trained_tree_num_nodes.argtypes = [ctypes.c_void_p]
        L.ffd_trained_tree_num_nodes.restype = ctypes.c_int64
        L.ffd_trained_tree_num_leaves.argtypes = [ctypes.c_void_p]
        L.ffd_trained_tree_num_leaves.restype = ctypes.c_int64
        L.ffd_trained_tree_arrays.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 9
        L.ffd_trained_tree_arrays.restype = ctypes.c_int
        L.ffd_trained_tree_stats.argtypes = [ctypes.c_void_p, P(_TrainStats)]
        L.ffd_trained_tree_stats.restype = ctypes.c_int
        L.ffd_trained_tree_archive.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, P(ctypes.c_int64)]
        L.ffd_trained_tree_archive.restype = ctypes.c_int
        L.ffd_trained_tree_save.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.ffd_trained_tree_save.restype = ctypes.c_int
        L.ffd_trained_tree_free.argtypes = [ctypes.c_void_p]
        L.ffd_train_hp_tree.argtypes = [P(_TrainParam), P(_TrainHpImage), ctypes.c_int32, P(ctypes.c_void_p)]
        L.ffd_train_hp_tree.restype = ctypes.c_int
        L.ffd_trained_tree_kind.argtypes = [ctypes.c_void_p]
        L.ffd_trained_tree_kind.restype = ctypes.c_int32
        L.ffd_trained_tree_num_samples.argtypes = [ctypes.c_void_p]
        L.ffd_trained_tree_num_samples.restype = ctypes.c_int64
        L.ffd_trained_tree_hp_arrays.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 8
        L.ffd_trained_tree_hp_arrays.restype = ctypes.c_int
        _bound = True
    return L


@dataclass
class ForestParam:                       # include/Constants.hpp:24-60 (data/config_ffd.txt values)
    max_depth: int = 20
    min_patches: int = 20
    ntests: int = 2500
    ntrees: int = 20
    nimages: int = 600
    npatches: int = 150
    face_size: int = 125
    patch_size_ratio: float = 0.25
    tree_path: str = "data/trees_ffd"
    image_path: str = "../../database/faces/lfw/lfw_ffd_ann.txt"

    @classmethod
    def headpose(cls, **kw):             # data/config_headpose.txt
        d = dict(max_depth=15, min_patches=20, ntests=2000, ntrees=15, nimages=400, npatches=200,
                 tree_path="data/trees_headpose")
        d.update(kw)
        return cls(**d)

    def getPatchSize(self):              # Constants.hpp:27-30
        return int(np.round(np.float32(self.face_size) * np.float32(self.patch_size_ratio)))


def _check(st):
    if st != 0:
        raise FFDError(st, _lib().ffd_train_last_error().decode())


class TrainedTree:
    """A grown Tree<MPSample> or Tree<HeadPoseSample>: pre-order node arrays (FFDMODEL layout), leaf
    payloads (MPLeaf / HeadPoseLeaf), the archive."""

    def __init__(self, handle):
        self._h = handle

    def __del__(self):
        self.close()

    def close(self):
        if getattr(self, "_h", None):
            _lib().ffd_trained_tree_free(self._h)
            self._h = None

    @property
    def num_nodes(self):
        return int(_lib().ffd_trained_tree_num_nodes(self._h))

    @property
    def num_leaves(self):
        return int(_lib().ffd_trained_tree_num_leaves(self._h))

    @property
    def kind(self):
        """0 = head pose (FFD_FOREST_HEADPOSE), 1 = facial features (FFD_FOREST_FFD)."""
        return int(_lib().ffd_trained_tree_kind(self._h))

    @property
    def num_samples(self):
        return int(_lib().ffd_trained_tree_num_samples(self._h))

    def arrays(self, n_samples=None, samples=None):
        """The tree's pre-order arrays.  The sampled training patches are included when `samples` is true
        (facial-feature trees; head-pose trees always include them); the buffer is sized from
        num_samples.  `n_samples` is accepted for compatibility and must equal num_samples when given."""
        n, l = self.num_nodes, self.num_leaves
        if n_samples is not None and n_samples != self.num_samples:
            raise ValueError(f"n_samples {n_samples} != num_samples {self.num_samples}")
        want = bool(samples) if samples is not None else bool(n_samples)
        if self.kind == 0:  # HeadPoseLeaf payloads, split modes, (image, x, y, label) patches
            a = {"node_leaf": np.zeros(n, np.int32), "node_split": np.zeros((n, 10), np.int16),
                 "node_info": np.zeros(n, np.float64), "node_mode": np.zeros(n, np.int32),
                 "leaf_n": np.zeros(l, np.int32), "leaf_fg": np.zeros(l, np.float32),
                 "leaf_labels": np.zeros((l, 5), np.int32), "samples": np.zeros((self.num_samples, 4), np.int32)}
            _check(_lib().ffd_trained_tree_hp_arrays(self._h, *(a[k].ctypes.data for k in
                   ("node_leaf", "node_split", "node_info", "node_mode", "leaf_n", "leaf_fg", "leaf_labels",
                    "samples"))))
            return a
        a = {"node_leaf": np.zeros(n, np.int32), "node_split": np.zeros((n, 10), np.int16),
             "node_info": np.zeros(n, np.float64), "leaf_n": np.zeros(l, np.int32), "leaf_fg": np.zeros(l, np.float32),
             "leaf_offset": np.zeros((l, 10, 2), np.int16), "leaf_var": np.zeros((l, 10), np.float32),
             "leaf_pf": np.zeros((l, 10), np.float32),
             "samples": np.zeros((self.num_samples if want else 0, 3), np.int32)}
        _check(_lib().ffd_trained_tree_arrays(self._h, *(a[k].ctypes.data for k in
               ("node_leaf", "node_split", "node_info", "leaf_n", "leaf_fg", "leaf_offset", "leaf_var", "leaf_pf")),
               a["samples"].ctypes.data if want else None))
        return a

    @property
    def stats(self):
        s = _TrainStats()
        _check(_lib().ffd_trained_tree_stats(self._h, ctypes.byref(s)))
        return {k: getattr(s, k) for k, _ in _TrainStats._fields_}

    def archive(self):
        """Tree<S>::save's bytes (Tree.hpp:239-256)."""
        size = ctypes.c_int64(0)
        _check(_lib().ffd_trained_tree_archive(self._h, None, 0, ctypes.byref(size)))
        buf = ctypes.create_string_buffer(size.value)
        _check(_lib().ffd_trained_tree_archive(self._h, buf, size.value, ctypes.byref(size)))
        return buf.raw[:size.value]

    def save(self, path):
        _check(_lib().ffd_trained_tree_save(self._h, str(path).encode()))


def train_mp_tree(rois, parts, param=None, tree_seed=1, split_seed=1, save_path="tree_000.txt", device=0):
    """trainTree (src/train_ffd.cpp:34-123) from the training ROIs: rois = list of uint8 gray images (the
    enlarged faces at face_size scale), parts = [n, 10, 2] landmarks in ROI pixels.  tree_seed is
    idx_tree + 1; split_seed stands for SplitGen::generateMT's std::time(NULL) (include/ffd.h)."""
    L = _lib()
    p = param or ForestParam()
    c = _TrainParam()
    L.ffd_train_param_init(ctypes.byref(c))
    for k in ("max_depth", "min_patches", "ntests", "ntrees", "nimages", "npatches", "face_size", "patch_size_ratio"):
        setattr(c, k, getattr(p, k))
    keep = [p.tree_path.encode(), p.image_path.encode(), str(save_path).encode()]
    c.tree_path, c.image_path, c.save_path = keep
    c.tree_seed, c.split_seed, c.device = tree_seed, split_seed, device
    parts = np.ascontiguousarray(parts, np.int32)
    rois = [np.ascontiguousarray(r, np.uint8) for r in rois]
    if len(rois) != len(parts) or parts.shape[1:] != (10, 2):
        raise ValueError("rois and parts [n, 10, 2] must match")
    imgs = (_TrainImage * len(rois))()
    for i, r in enumerate(rois):
        imgs[i].gray = r.ctypes.data
        imgs[i].height, imgs[i].width = r.shape
        imgs[i].stride = r.shape[1]
        imgs[i].parts = parts[i].ctypes.data
    h = ctypes.c_void_p()
    _check(L.ffd_train_mp_tree(ctypes.byref(c), imgs, len(rois), ctypes.byref(h)))
    return TrainedTree(h.value)


def train_hp_tree(images, faces, poses, param=None, tree_seed=1, split_seed=1,
                  save_path="data/trees_headpose/tree_000.txt", device=0):
    """train_headpose.cpp's trainTree (src/train_headpose.cpp:40-143) from the scaled images: images = list
    of uint8 gray images already scaled so the face box is face_size wide, faces = [n, 4] (x, y, w, h)
    boxes in them, poses = [n] head-pose classes in [-2, 2].  param defaults to config_headpose.txt."""
    L = _lib()
    p = param or ForestParam.headpose()
    c = _TrainParam()
    L.ffd_train_param_init(ctypes.byref(c))
    for k in ("max_depth", "min_patches", "ntests", "ntrees", "nimages", "npatches", "face_size", "patch_size_ratio"):
        setattr(c, k, getattr(p, k))
    keep = [p.tree_path.encode(), p.image_path.encode(), str(save_path).encode()]
    c.tree_path, c.image_path, c.save_path = keep
    c.tree_seed, c.split_seed, c.device = tree_seed, split_seed, device
    images = [np.ascontiguousarray(r, np.uint8) for r in images]
    faces = np.asarray(faces, np.int32).reshape(-1, 4)
    poses = np.asarray(poses, np.int32).reshape(-1)
    if not (len(images) == len(faces) == len(poses)):
        raise ValueError("images, faces [n, 4] and poses [n] must match")
    imgs = (_TrainHpImage * len(images))()
    for i, r in enumerate(images):
        imgs[i].gray = r.ctypes.data
        imgs[i].height, imgs[i].width = r.shape
        imgs[i].stride = r.shape[1]
        imgs[i].face = _Rect(*(int(v) for v in faces[i]))
        imgs[i].pose = int(poses[i])
    h = ctypes.c_void_p()
    _check(L.ffd_train_hp_tree(ctypes.byref(c), imgs, len(images), ctypes.byref(h)))
    return TrainedTree(h.value)
