"""ctypes wrapper for the CPU restatement (oracle/ffd_oracle.cpp).

TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package.  The product (the HIP engine behind
include/ffd.h) never links, calls or falls back to it.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libffd_oracle.so")
MAX_TREES = 32


class OracleFace(ctypes.Structure):
    _fields_ = [
        ("headpose", ctypes.c_float),
        ("pose_variance", ctypes.c_float),
        ("face_w", ctypes.c_int32),
        ("face_h", ctypes.c_int32),
        ("n_trees", ctypes.c_int32),
        ("points", (ctypes.c_int32 * 2) * 10),
    ]


class OracleTrace(ctypes.Structure):
    _fields_ = [
        ("face", ctypes.c_void_p),
        ("channels", ctypes.c_void_p),
        ("hp_leaves", ctypes.c_void_p),
        ("mp_leaves", ctypes.c_void_p),
        ("trees", ctypes.c_void_p),
        ("pose_freq", ctypes.c_void_p),
        ("vote_counts", ctypes.c_void_p),
        ("ms_mean", ctypes.c_void_p),
    ]


class OracleOptions(ctypes.Structure):
    """HeadPoseEstimatorOption / MultiPartEstimatorOption (FaceForest.hpp:34-58) + analyzeFace's
    MeanShiftOption (MeanShift.hpp:16-25); defaults = the reference constructors."""
    _fields_ = [("hp_num_labels", ctypes.c_int32), ("hp_step", ctypes.c_int32), ("hp_min_fg", ctypes.c_float),
                ("mp_num_parts", ctypes.c_int32), ("mp_step_x", ctypes.c_int32), ("mp_step_y", ctypes.c_int32),
                ("mp_min_samples", ctypes.c_int32), ("mp_min_fg", ctypes.c_float), ("mp_min_pf", ctypes.c_float),
                ("mp_max_var", ctypes.c_float), ("ms_kernel", ctypes.c_int32), ("ms_iter", ctypes.c_int32),
                ("ms_stop", ctypes.c_float)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle library missing: {LIB_PATH} (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_load_model.argtypes = [ctypes.c_char_p]
        L.oracle_set_steps.argtypes = [ctypes.c_int32] * 3
        L.oracle_set_options.argtypes = [ctypes.POINTER(OracleOptions)]
        L.oracle_get_options.argtypes = [ctypes.POINTER(OracleOptions)]
        L.oracle_last_error.restype = ctypes.c_char_p
        L.oracle_analyze_face.argtypes = [ctypes.c_void_p] + [ctypes.c_int32] * 8 + [
            ctypes.POINTER(OracleFace), ctypes.POINTER(OracleTrace)]
        L.oracle_face_geometry.argtypes = [ctypes.c_int32, ctypes.c_int32] + [ctypes.POINTER(ctypes.c_int32)] * 4
        L.oracle_bgr2gray.argtypes = [ctypes.c_void_p] + [ctypes.c_int32] * 3 + [ctypes.c_void_p]
        L.oracle_resize.argtypes = [ctypes.c_void_p] + [ctypes.c_int32] * 5 + [ctypes.c_void_p]
        L.oracle_channels.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
        L.oracle_gabor_kernel.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)]
        L.oracle_gabor_mag.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
        L.oracle_area_under_curve.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_double, ctypes.c_double]
        L.oracle_area_under_curve.restype = ctypes.c_double
        L.oracle_exp.argtypes = [ctypes.c_double]
        L.oracle_exp.restype = ctypes.c_double
        L.oracle_expf.argtypes = [ctypes.c_float]
        L.oracle_expf.restype = ctypes.c_float
        L.oracle_meanshift.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int32] * 3 + [ctypes.c_float,
                                                                                                   ctypes.c_void_p]
        L.oracle_estimate_headpose.argtypes = [ctypes.c_void_p] + [ctypes.c_int32] * 6 + [
            ctypes.POINTER(ctypes.c_float)] * 2
        L.oracle_estimate_facial_features.argtypes = [ctypes.c_void_p] + [ctypes.c_int32] * 6 + [
            ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
        L.oracle_detect_faces.argtypes = [ctypes.c_void_p] + [ctypes.c_int32] * 5 + [ctypes.c_float, ctypes.c_int32,
            ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), ctypes.c_void_p, ctypes.c_int32,
            ctypes.POINTER(ctypes.c_int32)]
        L.oracle_eval_patches.argtypes = [ctypes.c_void_p] + [ctypes.c_int32] * 3 + [ctypes.c_void_p, ctypes.c_int32,
                                                                                      ctypes.c_void_p, ctypes.c_int32,
                                                                                      ctypes.c_void_p]
        _lib = L
    return _lib


_loaded_model = None


def load_model(path):
    global _loaded_model
    if _loaded_model == path:
        return
    if lib().oracle_load_model(path.encode()) != 0:
        raise RuntimeError("oracle_load_model: " + lib().oracle_last_error().decode())
    _loaded_model = path


def set_steps(hp_step=4, mp_step_x=3, mp_step_y=3):
    """Patch-grid steps used by analyze_face / geometry (reference defaults 4, 3, 3)."""
    if lib().oracle_set_steps(hp_step, mp_step_x, mp_step_y) != 0:
        raise RuntimeError(lib().oracle_last_error().decode())


def get_options():
    o = OracleOptions()
    lib().oracle_get_options(ctypes.byref(o))
    return {k: getattr(o, k) for k, _ in OracleOptions._fields_}


def set_options(**kw):
    """Set estimator options (unnamed ones keep their current values); set_options() with no
    arguments is NOT a reset: use reset_options()."""
    cur = get_options()
    for k in kw:
        if k not in cur:
            raise KeyError(k)
    cur.update(kw)
    if lib().oracle_set_options(ctypes.byref(OracleOptions(**cur))) != 0:
        raise RuntimeError(lib().oracle_last_error().decode())


def reset_options():
    lib().oracle_set_options(None)


def _p(a):
    return a.ctypes.data if a is not None else None


def geometry(bw, bh):
    v = [ctypes.c_int32() for _ in range(4)]
    if lib().oracle_face_geometry(bw, bh, *[ctypes.byref(x) for x in v]) != 0:
        raise RuntimeError(lib().oracle_last_error().decode())
    return tuple(x.value for x in v)  # face_w, face_h, n_hp_patches, n_mp_patches


def analyze_face(img, bbox, threads=1, trace=False):
    """img: HxWx3 uint8 BGR; bbox (x, y, w, h). Returns (face dict, trace dict|None)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape[:2]
    x, y, bw, bh = [int(v) for v in bbox]
    out = OracleFace()
    tr = None
    bufs = None
    if trace:
        fw, fh, nhp, nmp = geometry(bw, bh)
        bufs = dict(
            face=np.zeros((fh, fw), np.uint8),
            channels=np.zeros((38, fh + 1, fw + 1), np.uint32),
            hp_leaves=np.zeros((nhp, 15), np.int32),
            mp_leaves=np.zeros(nmp * MAX_TREES, np.int32),
            trees=np.full(MAX_TREES, -1, np.int32),
            pose_freq=np.zeros(5, np.float32),
            vote_counts=np.zeros(10, np.int32),
            ms_mean=np.zeros((10, 2), np.float32),
        )
        tr = OracleTrace(*[_p(bufs[k]) for k, _ in OracleTrace._fields_])
    rc = lib().oracle_analyze_face(img.ctypes.data, w, h, img.strides[0], x, y, bw, bh, threads,
                                   ctypes.byref(out), ctypes.byref(tr) if tr is not None else None)
    if rc != 0:
        raise RuntimeError("oracle_analyze_face: " + lib().oracle_last_error().decode())
    face = dict(headpose=out.headpose, pose_variance=out.pose_variance, face_w=out.face_w,
                face_h=out.face_h, n_trees=out.n_trees,
                points=np.array([[out.points[i][0], out.points[i][1]] for i in range(10)], np.int32))
    if bufs is not None:
        nt = out.n_trees
        bufs["mp_leaves"] = bufs["mp_leaves"][: bufs["mp_leaves"].size // MAX_TREES * nt].reshape(-1, nt)
        bufs["trees"] = bufs["trees"][:nt]
    return face, bufs


def bgr2gray(img):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape[:2]
    out = np.zeros((h, w), np.uint8)
    lib().oracle_bgr2gray(img.ctypes.data, w, h, img.strides[0], out.ctypes.data)
    return out


def detect_faces(img, min_size=30, min_neighbors=1, scale_factor=1.3, widen=True, raw=False):
    """FaceForest::detectFace (src/FaceForest.cpp:136-159) restated: (boxes [n, 4] x, y, w, h) and,
    with raw=True, also the ungrouped candidates in scan order.  Parity with OpenCV unpinned."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape[:2]
    cap = 4096
    for _ in range(3):
        boxes = np.zeros((cap, 4), np.int32)
        rawv = np.zeros((cap * 8, 4), np.int32)
        n, nr = ctypes.c_int32(), ctypes.c_int32()
        if lib().oracle_detect_faces(img.ctypes.data, w, h, img.strides[0], min_size, min_neighbors,
                                     scale_factor, int(widen), boxes.ctypes.data, cap, ctypes.byref(n),
                                     rawv.ctypes.data, cap * 8, ctypes.byref(nr)) != 0:
            raise RuntimeError(lib().oracle_last_error().decode())
        if n.value <= cap and nr.value <= cap * 8:
            break
        cap = max(n.value, nr.value // 8 + 1)
    out = boxes[: n.value].copy()
    return (out, rawv[: nr.value].copy()) if raw else out


def resize(src, dw, dh):
    src = np.ascontiguousarray(src, np.uint8)
    out = np.zeros((dh, dw), np.uint8)
    lib().oracle_resize(src.ctypes.data, src.shape[1], src.shape[0], src.strides[0], dw, dh, out.ctypes.data)
    return out


def channels(face):
    face = np.ascontiguousarray(face, np.uint8)
    h, w = face.shape
    out = np.zeros((38, h + 1, w + 1), np.uint32)
    if lib().oracle_channels(face.ctypes.data, w, h, out.ctypes.data) != 0:
        raise RuntimeError(lib().oracle_last_error().decode())
    return out


def gabor_kernel(index):
    w = ctypes.c_int32()
    re = np.zeros(25 * 25, np.float32)
    im = np.zeros(25 * 25, np.float32)
    if lib().oracle_gabor_kernel(index, re.ctypes.data, im.ctypes.data, ctypes.byref(w)) != 0:
        raise RuntimeError(lib().oracle_last_error().decode())
    n = w.value
    return re[: n * n].reshape(n, n), im[: n * n].reshape(n, n)


def gabor_mag(face, index):
    face = np.ascontiguousarray(face, np.uint8)
    h, w = face.shape
    out = np.zeros((h, w), np.float32)
    lib().oracle_gabor_mag(face.ctypes.data, w, h, index, out.ctypes.data)
    return out


def area_under_curve(x1, x2, mean, std):
    return lib().oracle_area_under_curve(x1, x2, mean, std)


def meanshift(xy, w, kernel=10, iters=7, stop=0.05):
    """MeanShift::shift (MeanShift.hpp:41-135) of one vote list: the mode (x, y) before cvRound."""
    xy = np.ascontiguousarray(xy, np.int32).reshape(-1, 2)
    w = np.ascontiguousarray(w, np.float32)
    out = np.zeros(2, np.float32)
    lib().oracle_meanshift(xy.ctypes.data, w.ctypes.data, len(w), kernel, iters, stop, out.ctypes.data)
    return out


def exp(x):
    return lib().oracle_exp(x)


def expf(x):
    return lib().oracle_expf(x)


def eval_patches(channels, xy, kind, tree_ids):
    """Tree<S>::evaluateMT for a patch list: [n_patches][n_trees] leaf ordinals (kind 0 head pose, 1 FFD)."""
    ch = np.ascontiguousarray(channels, np.uint32)
    _, h1, w1 = ch.shape
    p = np.ascontiguousarray(xy, np.int32).reshape(-1, 2)
    t = np.ascontiguousarray(tree_ids, np.int32)
    out = np.zeros((p.shape[0], t.size), np.int32)
    if lib().oracle_eval_patches(ch.ctypes.data, w1 - 1, h1 - 1, int(kind), p.ctypes.data, p.shape[0], t.ctypes.data,
                                 t.size, out.ctypes.data) != 0:
        raise RuntimeError(lib().oracle_last_error().decode())
    return out


def estimate_headpose(channels, region=None):
    """FaceForest::estimateHeadPose on 38 integral planes (38 x (H+1) x (W+1)); region (x, y, w, h)."""
    ch = np.ascontiguousarray(channels, np.uint32)
    h, w = ch.shape[1] - 1, ch.shape[2] - 1
    rx, ry, rw, rh = region or (0, 0, w, h)
    hp, var = ctypes.c_float(), ctypes.c_float()
    if lib().oracle_estimate_headpose(ch.ctypes.data, w, h, rx, ry, rw, rh, ctypes.byref(hp), ctypes.byref(var)) != 0:
        raise RuntimeError(lib().oracle_last_error().decode())
    return hp.value, var.value


def estimate_facial_features(channels, region, tree_ids):
    """FaceForest::estimateFacialFeatures: 10 x 2 int landmarks in sample coordinates."""
    ch = np.ascontiguousarray(channels, np.uint32)
    h, w = ch.shape[1] - 1, ch.shape[2] - 1
    rx, ry, rw, rh = region or (0, 0, w, h)
    t = np.ascontiguousarray(tree_ids, np.int32)
    pts = np.zeros((10, 2), np.int32)
    if lib().oracle_estimate_facial_features(ch.ctypes.data, w, h, rx, ry, rw, rh, t.ctypes.data, t.size,
                                             pts.ctypes.data) != 0:
        raise RuntimeError(lib().oracle_last_error().decode())
    return pts


class OracleTrainParam(ctypes.Structure):
    """ForestParam (Constants.hpp:24-60) + the seeds (oracle/ffd_oracle.h oracle_train_param)."""
    _fields_ = [("max_depth", ctypes.c_int32), ("min_patches", ctypes.c_int32), ("ntests", ctypes.c_int32),
                ("ntrees", ctypes.c_int32), ("nimages", ctypes.c_int32), ("npatches", ctypes.c_int32),
                ("face_size", ctypes.c_int32), ("patch_size_ratio", ctypes.c_float),
                ("num_thresholds", ctypes.c_int32), ("tree_seed", ctypes.c_uint32), ("split_seed", ctypes.c_uint32),
                ("lamda", ctypes.c_float)]


def train_mp_tree(rois, parts, max_depth=20, min_patches=20, ntests=2500, npatches=150, face_size=125,
                  patch_size_ratio=0.25, tree_seed=1, split_seed=1, ntrees=20, nimages=600):
    """The CPU restatement of trainTree + Tree<MPSample> growth (oracle/ffd_train_oracle.cpp): returns the
    pre-order node arrays, MPLeaf payloads, sampled patches and i_node."""
    L = lib()
    if not getattr(L, "_train_bound", False):
        L.oracle_train_mp_tree.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(OracleTrainParam),
                                           ctypes.POINTER(ctypes.c_void_p)]
        L.oracle_train_tree_size.argtypes = [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_int64)] * 3
        L.oracle_train_tree_get.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 9
        L.oracle_train_tree_free.argtypes = [ctypes.c_void_p]
        L.oracle_train_last_error.restype = ctypes.c_char_p
        L.oracle_log.argtypes = [ctypes.c_double]
        L.oracle_log.restype = ctypes.c_double
        L._train_bound = True
    rois = [np.ascontiguousarray(r, np.uint8) for r in rois]
    parts = np.ascontiguousarray(parts, np.int32)
    n = len(rois)
    ptrs = (ctypes.c_void_p * n)(*[r.ctypes.data for r in rois])
    ws = np.array([r.shape[1] for r in rois], np.int32)
    hs = np.array([r.shape[0] for r in rois], np.int32)
    p = OracleTrainParam(max_depth, min_patches, ntests, ntrees, nimages, npatches, face_size, patch_size_ratio,
                         25, tree_seed, split_seed, 0.125)
    h = ctypes.c_void_p()
    if L.oracle_train_mp_tree(ptrs, ws.ctypes.data, hs.ctypes.data, parts.ctypes.data, n, parts.shape[1],
                              ctypes.byref(p), ctypes.byref(h)) != 0:
        raise RuntimeError("oracle_train_mp_tree: " + L.oracle_train_last_error().decode())
    try:
        nn, nl, inode = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        L.oracle_train_tree_size(h, ctypes.byref(nn), ctypes.byref(nl), ctypes.byref(inode))
        N, Lf = nn.value, nl.value
        a = {"node_leaf": np.zeros(N, np.int32), "node_split": np.zeros((N, 10), np.int16),
             "node_info": np.zeros(N, np.float64), "leaf_n": np.zeros(Lf, np.int32), "leaf_fg": np.zeros(Lf, np.float32),
             "leaf_offset": np.zeros((Lf, 10, 2), np.int16), "leaf_var": np.zeros((Lf, 10), np.float32),
             "leaf_pf": np.zeros((Lf, 10), np.float32), "samples": np.zeros((n * npatches, 3), np.int32)}
        L.oracle_train_tree_get(h, *(a[k].ctypes.data for k in ("node_leaf", "node_split", "node_info", "leaf_n",
                                                                 "leaf_fg", "leaf_offset", "leaf_var", "leaf_pf",
                                                                 "samples")))
        a["i_node"] = inode.value
        return a
    finally:
        L.oracle_train_tree_free(h)


def train_hp_tree(images, faces, poses, max_depth=15, min_patches=20, ntests=2000, npatches=200, face_size=125,
                  patch_size_ratio=0.25, tree_seed=1, split_seed=1, ntrees=15, nimages=400):
    """The CPU restatement of train_headpose.cpp's trainTree + Tree<HeadPoseSample> growth
    (oracle/ffd_train_oracle.cpp): images already scaled so the face box is face_size wide, faces
    [n, 4] (x, y, w, h), poses [n] in [-2, 2].  Returns the pre-order node arrays, the split modes,
    HeadPoseLeaf payloads, the sampled patches (image, x, y, label) and i_node."""
    L = lib()
    if not getattr(L, "_train_hp_bound", False):
        L.oracle_train_hp_tree.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int32, ctypes.POINTER(OracleTrainParam),
                                                                   ctypes.POINTER(ctypes.c_void_p)]
        L.oracle_train_hp_tree_size.argtypes = [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_int64)] * 4
        L.oracle_train_hp_tree_get.argtypes = [ctypes.c_void_p] * 9
        L.oracle_train_hp_tree_free.argtypes = [ctypes.c_void_p]
        L.oracle_train_last_error.restype = ctypes.c_char_p
        L._train_hp_bound = True
    images = [np.ascontiguousarray(r, np.uint8) for r in images]
    faces = np.ascontiguousarray(faces, np.int32).reshape(-1, 4)
    poses = np.ascontiguousarray(poses, np.int32)
    n = len(images)
    ptrs = (ctypes.c_void_p * n)(*[r.ctypes.data for r in images])
    ws = np.array([r.shape[1] for r in images], np.int32)
    hs = np.array([r.shape[0] for r in images], np.int32)
    p = OracleTrainParam(max_depth, min_patches, ntests, ntrees, nimages, npatches, face_size, patch_size_ratio,
                         25, tree_seed, split_seed, 0.125)
    h = ctypes.c_void_p()
    if L.oracle_train_hp_tree(ptrs, ws.ctypes.data, hs.ctypes.data, faces.ctypes.data, poses.ctypes.data, n,
                              ctypes.byref(p), ctypes.byref(h)) != 0:
        raise RuntimeError("oracle_train_hp_tree: " + L.oracle_train_last_error().decode())
    try:
        nn, nl, inode, ns = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        L.oracle_train_hp_tree_size(h, ctypes.byref(nn), ctypes.byref(nl), ctypes.byref(inode), ctypes.byref(ns))
        N, Lf = nn.value, nl.value
        a = {"node_leaf": np.zeros(N, np.int32), "node_split": np.zeros((N, 10), np.int16),
             "node_info": np.zeros(N, np.float64), "node_mode": np.zeros(N, np.int32), "leaf_n": np.zeros(Lf, np.int32),
             "leaf_fg": np.zeros(Lf, np.float32), "leaf_labels": np.zeros((Lf, 5), np.int32),
             "samples": np.zeros((ns.value, 4), np.int32)}
        L.oracle_train_hp_tree_get(h, *(a[k].ctypes.data for k in ("node_leaf", "node_split", "node_info", "node_mode",
                                                                    "leaf_n", "leaf_fg", "leaf_labels", "samples")))
        a["i_node"] = inode.value
        return a
    finally:
        L.oracle_train_hp_tree_free(h)


def log(x):
    lib()
    if not getattr(lib(), "_train_bound", False):
        lib().oracle_log.argtypes = [ctypes.c_double]
        lib().oracle_log.restype = ctypes.c_double
    return lib().oracle_log(x)
