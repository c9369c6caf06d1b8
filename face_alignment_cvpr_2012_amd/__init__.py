"""MI355X-native conditional-regression-forest facial-landmark engine.

Python host mirror of the reference's public API over the C-ABI in include/ffd.h
(libffd.so, HIP kernels for gfx950).  Names follow the reference
(/root/reference/include/FaceForest.hpp): FaceForestOptions, Face, FaceForest with
analyzeFace / analyzeImage, and Forest.evaluate (Forest<S>::evaluateMT,
include/Forest.hpp:80-90).

The product path is the HIP engine only: if libffd.so is missing or no HIP
device is usable, construction raises (there is no CPU fallback; the CPU
restatement in oracle/ is test infrastructure).
"""
import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

__all__ = [
    "FaceForestOptions", "HeadPoseEstimatorOption", "MultiPartEstimatorOption", "MeanShiftOption",
    "Face", "FaceForest", "FaceForestGroup", "Forest", "FFDError", "default_model_path", "library_path",
    "comm_id", "status_string", "ImageSample", "meanshift",
    "FOREST_HEADPOSE", "FOREST_FFD", "LANDMARK_NAMES",
]

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
FOREST_HEADPOSE = 0
FOREST_FFD = 1
MAX_TREES = 32
NUM_CHANNELS = 38
LANDMARK_NAMES = ("left eye (l)", "left eye (r)", "mouth (l)", "mouth (r)", "mouth (b)", "mouth (t)",
                  "right eye (l)", "right eye (r)", "nose (l)", "nose (r)")  # output/generate_report.m:13-15


def library_path():
    return os.environ.get("FFD_LIBRARY") or os.path.join(HERE, "lib", "libffd.so")  # (an empty value: the in-tree one)


def default_model_path():
    return os.environ.get("FFD_MODEL", os.path.join(REPO, "model", "ffd_model.bin"))


class FFDError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"ffd status {status}: {msg}")
        self.status = status


# ------------------------------------------------------------------ ctypes --
class _Rect(ctypes.Structure):
    _fields_ = [("x", ctypes.c_int32), ("y", ctypes.c_int32), ("width", ctypes.c_int32), ("height", ctypes.c_int32)]


class _Image(ctypes.Structure):
    _fields_ = [("bgr", ctypes.c_void_p), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("stride", ctypes.c_int32)]


class _Face(ctypes.Structure):
    _fields_ = [("headpose", ctypes.c_float), ("pose_variance", ctypes.c_float), ("bbox", _Rect),
                ("points", (ctypes.c_int32 * 2) * 10), ("n_trees", ctypes.c_int32), ("status", ctypes.c_int32)]


FACE_RECORD_BYTES = ctypes.sizeof(_Face)


class _HpOpt(ctypes.Structure):
    _fields_ = [("num_head_pose_labels", ctypes.c_int32), ("step_size", ctypes.c_int32),
                ("min_foreground_probability", ctypes.c_float)]


class _MpOpt(ctypes.Structure):
    _fields_ = [("num_parts", ctypes.c_int32), ("step_size", ctypes.c_int32), ("min_samples", ctypes.c_int32),
                ("min_forground", ctypes.c_float), ("min_pf", ctypes.c_float), ("max_variance", ctypes.c_float),
                ("step_size_y", ctypes.c_int32)]


class _MsOpt(ctypes.Structure):
    _fields_ = [("kernel_size", ctypes.c_int32), ("max_iterations", ctypes.c_int32),
                ("stopping_criteria", ctypes.c_float)]


class _Desc(ctypes.Structure):
    _fields_ = [("model_path", ctypes.c_char_p), ("device", ctypes.c_int32), ("max_chunk_faces", ctypes.c_int32),
                ("hp_option", _HpOpt), ("mp_option", _MpOpt), ("ms_option", _MsOpt)]


class _HpLeaf(ctypes.Structure):          # ffd_headpose_leaf = HeadPoseLeaf (HeadPoseSample.hpp:144-162)
    _fields_ = [("hp_nsamples", ctypes.c_int32), ("hp_foreground", ctypes.c_float), ("hp_labels", ctypes.c_int32 * 5)]


class _MpLeaf(ctypes.Structure):          # ffd_mp_leaf = MPLeaf (MPSample.hpp:137-159)
    _fields_ = [("mp_samples", ctypes.c_int32), ("mp_foreground", ctypes.c_float),
                ("mp_parts_offset", (ctypes.c_int32 * 2) * 10), ("mp_parts_variance", ctypes.c_float * 10),
                ("mp_prob_foreground", ctypes.c_float * 10)]


class _DetOpt(ctypes.Structure):
    _fields_ = [("min_feature_size", ctypes.c_int32), ("min_neighbors", ctypes.c_int32),
                ("search_scale_factor", ctypes.c_float), ("widen", ctypes.c_int32)]


class _Trace(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in
                ("face", "channels", "hp_leaves", "mp_leaves", "trees", "pose_freq", "vote_counts", "ms_mean")]


_lib = None

# Every symbol include/ffd.h declares (tests check the library exports them all).
EXPORTED_SYMBOLS = (
    "ffd_engine_desc_init", "ffd_engine_create", "ffd_engine_destroy", "ffd_last_error", "ffd_face_geometry",
    "ffd_analyze_faces", "ffd_analyze_faces_device", "ffd_synchronize", "ffd_stream", "ffd_extract_channels",
    "ffd_forest_eval_leaves", "ffd_get_trace", "ffd_version", "ffd_set_profiling", "ffd_get_stage_times", "ffd_check_mag_sqrt",
    "ffd_stage_name", "ffd_status_string", "ffd_estimate_headpose", "ffd_estimate_facial_features", "ffd_forest_leaves",
    "ffd_group_create", "ffd_group_destroy", "ffd_group_last_error", "ffd_group_size", "ffd_group_engine",
    "ffd_group_analyze_faces", "ffd_comm_id", "ffd_engine_join", "ffd_gather_faces", "ffd_engine_comm_info",
    "ffd_detect_options_init", "ffd_detect_faces", "ffd_detect_faces_device", "ffd_analyze_images",
    "ffd_detect_candidates", "ffd_detector_create", "ffd_model_open", "ffd_model_close", "ffd_model_last_error", "ffd_model_num_trees", "ffd_model_tree_save_path",
    "ffd_model_tree_archive", "ffd_model_save_tree",
    "ffd_train_param_init", "ffd_train_mp_tree", "ffd_train_mp_tree_patches", "ffd_train_last_error", "ffd_trained_tree_num_nodes",
    "ffd_trained_tree_num_leaves", "ffd_trained_tree_arrays", "ffd_trained_tree_stats", "ffd_trained_tree_archive",
    "ffd_trained_tree_save", "ffd_trained_tree_free",
    "ffd_train_hp_param_init", "ffd_train_hp_tree", "ffd_trained_tree_kind", "ffd_trained_tree_num_samples",
    "ffd_trained_tree_hp_arrays",
    "ffd_sample_create", "ffd_sample_create_from_channels", "ffd_sample_destroy", "ffd_sample_size",
    "ffd_sample_channels", "ffd_sample_eval_leaves", "ffd_sample_eval_grid", "ffd_sample_estimate_headpose",
    "ffd_sample_estimate_facial_features", "ffd_meanshift", "ffd_model_convert", "ffd_model_convert_last_error",
    "ffd_forest_subdirs", "ffd_group_debug_overlap", "ffd_forest_tree_leaves",
)
COMM_ID_BYTES = 128
STATUS_OK, STATUS_INVALID_ARGUMENT, STATUS_OUT_OF_MEMORY, STATUS_UNSUPPORTED = 0, 1, 4, 7
NUM_STAGES = 12


def lib():
    """Load libffd.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if not os.path.exists(path):
        raise FFDError(-1, f"HIP engine library not built: {path} (run __graft_entry__.build())")
    L = ctypes.CDLL(path)
    P = ctypes.POINTER
    L.ffd_engine_desc_init.argtypes = [P(_Desc)]
    L.ffd_engine_create.argtypes = [P(_Desc), P(ctypes.c_void_p)]
    L.ffd_engine_destroy.argtypes = [ctypes.c_void_p]
    L.ffd_last_error.argtypes = [ctypes.c_void_p]
    L.ffd_last_error.restype = ctypes.c_char_p
    L.ffd_version.restype = ctypes.c_char_p
    L.ffd_face_geometry.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32] + [P(ctypes.c_int32)] * 4
    L.ffd_analyze_faces.argtypes = [ctypes.c_void_p, P(_Image), ctypes.c_int32, P(_Rect), ctypes.c_void_p,
                                    ctypes.c_int32, P(_Face)]
    L.ffd_analyze_faces_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                           ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
    L.ffd_synchronize.argtypes = [ctypes.c_void_p]
    L.ffd_stream.argtypes = [ctypes.c_void_p]
    L.ffd_stream.restype = ctypes.c_void_p
    L.ffd_extract_channels.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_void_p]
    L.ffd_forest_eval_leaves.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                         ctypes.c_int32, ctypes.c_void_p]
    L.ffd_get_trace.argtypes = [ctypes.c_void_p, ctypes.c_int32, P(_Trace)]
    L.ffd_set_profiling.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L.ffd_get_stage_times.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
    L.ffd_stage_name.argtypes = [ctypes.c_int32]
    L.ffd_stage_name.restype = ctypes.c_char_p
    L.ffd_check_mag_sqrt.argtypes = [ctypes.c_void_p, P(ctypes.c_uint64), P(ctypes.c_uint64)]
    L.ffd_status_string.argtypes = [ctypes.c_int32]
    L.ffd_status_string.restype = ctypes.c_char_p
    L.ffd_estimate_headpose.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                        P(_Rect), P(_HpOpt), P(ctypes.c_float), P(ctypes.c_float)]
    L.ffd_estimate_facial_features.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                               P(_Rect), ctypes.c_void_p, ctypes.c_int32, P(_MpOpt), ctypes.c_void_p]
    L.ffd_forest_leaves.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
    L.ffd_group_create.argtypes = [P(_Desc), ctypes.c_void_p, ctypes.c_int32, P(ctypes.c_void_p)]
    L.ffd_group_destroy.argtypes = [ctypes.c_void_p]
    L.ffd_group_last_error.argtypes = [ctypes.c_void_p]
    L.ffd_group_last_error.restype = ctypes.c_char_p
    L.ffd_group_size.argtypes = [ctypes.c_void_p]
    L.ffd_group_engine.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L.ffd_group_engine.restype = ctypes.c_void_p
    L.ffd_group_analyze_faces.argtypes = [ctypes.c_void_p, P(_Image), ctypes.c_int32, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_int32, P(_Face)]
    L.ffd_comm_id.argtypes = [ctypes.c_void_p]
    L.ffd_engine_join.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
    L.ffd_gather_faces.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]
    L.ffd_engine_comm_info.argtypes = [ctypes.c_void_p, P(ctypes.c_int32), P(ctypes.c_int32)]
    L.ffd_detect_options_init.argtypes = [P(_DetOpt)]
    L.ffd_detect_faces.argtypes = [ctypes.c_void_p, P(_Image), ctypes.c_int32, P(_DetOpt), ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_int32, P(ctypes.c_int32)]
    L.ffd_detect_faces_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                          ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, P(_DetOpt), ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_int32, P(ctypes.c_int32)]
    L.ffd_analyze_images.argtypes = [ctypes.c_void_p, P(_Image), ctypes.c_int32, P(_DetOpt), ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_int32, P(ctypes.c_int32)]
    L.ffd_detect_candidates.argtypes = [ctypes.c_void_p, P(_Image), P(_DetOpt), ctypes.c_void_p, ctypes.c_int32,
                                        P(ctypes.c_int32)]
    L.ffd_model_open.argtypes = [ctypes.c_char_p, P(ctypes.c_void_p)]
    L.ffd_model_close.argtypes = [ctypes.c_void_p]
    L.ffd_model_last_error.restype = ctypes.c_char_p
    L.ffd_model_num_trees.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L.ffd_model_num_trees.restype = ctypes.c_int32
    L.ffd_model_tree_save_path.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p,
                                           ctypes.c_int32]
    L.ffd_model_tree_archive.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                         ctypes.c_int64, P(ctypes.c_int64)]
    L.ffd_model_save_tree.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p]
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    L.ffd_sample_create.argtypes = [vp, vp, i32, i32, i32, P(vp)]
    L.ffd_sample_create_from_channels.argtypes = [vp, vp, i32, i32, P(vp)]
    L.ffd_sample_destroy.argtypes = [vp]
    L.ffd_sample_destroy.restype = None
    L.ffd_sample_size.argtypes = [vp, P(i32), P(i32)]
    L.ffd_sample_channels.argtypes = [vp, vp]
    L.ffd_sample_eval_leaves.argtypes = [vp, i32, vp, i32, vp, i32, vp]
    L.ffd_sample_eval_grid.argtypes = [vp, i32, i32, i32, i32, i32, i32, vp, i32, vp]
    L.ffd_sample_estimate_headpose.argtypes = [vp, P(_Rect), P(_HpOpt), P(ctypes.c_float), P(ctypes.c_float)]
    L.ffd_sample_estimate_facial_features.argtypes = [vp, P(_Rect), vp, i32, P(_MpOpt), vp]
    L.ffd_meanshift.argtypes = [vp, vp, i32, P(_MsOpt), vp]
    L.ffd_model_convert_last_error.restype = ctypes.c_char_p
    L.ffd_group_debug_overlap.argtypes = [i32, i32, P(ctypes.c_double)]
    L.ffd_group_debug_overlap.restype = ctypes.c_int
    for name in ("ffd_sample_create", "ffd_sample_create_from_channels", "ffd_sample_size", "ffd_sample_channels",
                 "ffd_sample_eval_leaves", "ffd_sample_eval_grid", "ffd_sample_estimate_headpose",
                 "ffd_sample_estimate_facial_features", "ffd_meanshift"):
        getattr(L, name).restype = ctypes.c_int
    for name in ("ffd_detect_faces", "ffd_detect_faces_device", "ffd_analyze_images", "ffd_detect_candidates",
                 "ffd_model_open", "ffd_model_tree_save_path", "ffd_model_tree_archive", "ffd_model_save_tree","ffd_engine_create", "ffd_face_geometry", "ffd_analyze_faces", "ffd_analyze_faces_device",
                 "ffd_synchronize", "ffd_extract_channels", "ffd_forest_eval_leaves", "ffd_get_trace",
                 "ffd_set_profiling", "ffd_get_stage_times", "ffd_estimate_headpose",
                 "ffd_estimate_facial_features", "ffd_forest_leaves", "ffd_group_create", "ffd_group_analyze_faces", "ffd_comm_id",
                 "ffd_engine_join", "ffd_gather_faces", "ffd_engine_comm_info", "ffd_group_size"):
        getattr(L, name).restype = ctypes.c_int
    _lib = L
    return L


# ----------------------------------------------------------------- options --
@dataclass
class HeadPoseEstimatorOption:          # include/FaceForest.hpp:34-43
    num_head_pose_labels: int = 5
    step_size: int = 4
    min_foreground_probability: float = 0.5


@dataclass
class MultiPartEstimatorOption:         # include/FaceForest.hpp:45-58
    num_parts: int = 10
    step_size: int = 3
    min_samples: int = 2
    min_forground: float = 0.5
    min_pf: float = 0.25
    max_variance: float = 25.0
    step_size_y: int = 0                # 0: step_size on both axes (the reference); C4 uses (2, 1)


@dataclass
class MeanShiftOption:                  # include/MeanShift.hpp:16-25
    kernel_size: int = 10
    max_iterations: int = 7
    stopping_criteria: float = 0.05


@dataclass
class FaceDetectionOption:              # include/FaceForest.hpp:21-32
    min_feature_size: int = 30
    min_neighbors: int = 1
    search_scale_factor: float = 1.3
    widen: bool = True                  # detectFace's 5 % / 15 % enlargement (FaceForest.cpp:148-158)


def _det_opt(o):
    o = o or FaceDetectionOption()
    return _DetOpt(int(o.min_feature_size), int(o.min_neighbors), float(o.search_scale_factor), int(bool(o.widen)))


@dataclass
class FaceForestOptions:                # include/FaceForest.hpp:60-68
    model_path: str = field(default_factory=default_model_path)
    device: int = 0
    max_chunk_faces: int = 0
    hp_option: HeadPoseEstimatorOption = field(default_factory=HeadPoseEstimatorOption)
    mp_option: MultiPartEstimatorOption = field(default_factory=MultiPartEstimatorOption)
    ms_option: MeanShiftOption = field(default_factory=MeanShiftOption)
    fd_option: FaceDetectionOption = field(default_factory=FaceDetectionOption)


@dataclass
class Face:                             # include/FaceForest.hpp:70-75
    headpose: float
    bbox: tuple
    ffd_cordinates: np.ndarray          # 10 x 2 int, bbox-relative
    pose_variance: float = 0.0
    n_trees: int = 0
    status: int = 0


def _face_from_record(r):
    return Face(headpose=float(r.headpose), bbox=(r.bbox.x, r.bbox.y, r.bbox.width, r.bbox.height),
                ffd_cordinates=np.array([[r.points[i][0], r.points[i][1]] for i in range(10)], np.int32),
                pose_variance=float(r.pose_variance), n_trees=int(r.n_trees), status=int(r.status))


def faces_from_records(buf):
    """Decode a bytes/uint8 buffer of ffd_face records (e.g. copied back from the device)."""
    arr = (_Face * (len(buf) // FACE_RECORD_BYTES)).from_buffer_copy(bytes(buf))
    return [_face_from_record(r) for r in arr]


def _packed_rects(boxes):
    """(n, 4) C-contiguous int32 view/copy of `boxes` (ffd_rect array layout)."""
    a = boxes if isinstance(boxes, np.ndarray) else np.asarray(boxes)
    a = np.ascontiguousarray(a, np.int32).reshape(-1, 4)
    return a


def _check(status, handle=None):
    if status != 0:
        msg = lib().ffd_last_error(handle).decode(errors="replace")
        raise FFDError(status, msg)


def _make_desc(o):
    """ffd_engine_desc from FaceForestOptions (returns the desc and the bytes its path points to)."""
    d = _Desc()
    lib().ffd_engine_desc_init(ctypes.byref(d))
    path = os.fspath(o.model_path).encode()
    d.model_path = path
    d.device = o.device
    d.max_chunk_faces = o.max_chunk_faces
    d.hp_option = _HpOpt(o.hp_option.num_head_pose_labels, o.hp_option.step_size, o.hp_option.min_foreground_probability)
    d.mp_option = _MpOpt(o.mp_option.num_parts, o.mp_option.step_size, o.mp_option.min_samples,
                         o.mp_option.min_forground, o.mp_option.min_pf, o.mp_option.max_variance,
                         o.mp_option.step_size_y)
    d.ms_option = _MsOpt(o.ms_option.kernel_size, o.ms_option.max_iterations, o.ms_option.stopping_criteria)
    return d, path


def status_string(status):
    return lib().ffd_status_string(int(status)).decode()


def _image_array(images):
    imgs = [np.ascontiguousarray(im, dtype=np.uint8) for im in images]
    cim = (_Image * len(imgs))()
    for i, im in enumerate(imgs):
        if im.ndim != 3 or im.shape[2] != 3:
            raise ValueError("images must be HxWx3 BGR uint8")
        cim[i] = _Image(im.ctypes.data, im.shape[1], im.shape[0], im.strides[0])
    return imgs, cim


# --------------------------------------------------------------- FaceForest --
class FaceForest:
    """FaceForest (include/FaceForest.hpp:81-157) on one MI355X device.

    One engine serves one caller at a time (include/ffd.h; the reference's analyzeFace is not reentrant
    either), and this object, its ImageSamples and Forests take no lock (the C++ header does): Python threads
    use one FaceForest each, or a FaceForestGroup (one host thread per device)."""

    def __init__(self, options=None):
        self.options = options or FaceForestOptions()
        L = lib()
        d, self._model_path_bytes = _make_desc(self.options)
        h = ctypes.c_void_p()
        st = L.ffd_engine_create(ctypes.byref(d), ctypes.byref(h))
        if st != 0:
            raise FFDError(st, L.ffd_last_error(None).decode(errors="replace"))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().ffd_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    # ---- reference API ------------------------------------------------------
    def analyzeFace(self, img, face_bbox):
        """FaceForest::analyzeFace(img, bbox, face) (src/FaceForest.cpp:183-258)."""
        return self.analyzeFaces([img], [face_bbox])[0]

    def analyzeImage(self, img, faces_bboxes=None):
        """FaceForest::analyzeImage (src/FaceForest.cpp:161-181): the GPU Haar detector
        (detectFace) then analyzeFace on every box.  With faces_bboxes given, those boxes are analysed
        instead (a caller-side detector)."""
        if faces_bboxes is not None:
            return self.analyzeFaces([img], list(faces_bboxes), [0] * len(faces_bboxes))
        return self.analyzeImages([img])[0]

    def detectFace(self, img, fd_option=None):
        """FaceForest::detectFace (src/FaceForest.cpp:136-159) on the GPU: boxes as (n, 4) int32."""
        return self.detectFaces([img], fd_option)[0]

    def detectFaces(self, images, fd_option=None):
        """detectFace over a batch of frames (one GPU pass); a list of (n_k, 4) arrays."""
        imgs, cim = _image_array(images)
        opt = _det_opt(fd_option or self.options.fd_option)
        cap = 64 * max(1, len(imgs))
        for _ in range(2):
            boxes = np.zeros((cap, 4), np.int32)
            owner = np.zeros(cap, np.int32)
            n = ctypes.c_int32()
            _check(lib().ffd_detect_faces(self._h, cim, len(imgs), ctypes.byref(opt), boxes.ctypes.data,
                                          owner.ctypes.data, cap, ctypes.byref(n)), self._h)
            if n.value <= cap:
                break
            cap = n.value
        return [boxes[: n.value][owner[: n.value] == k] for k in range(len(imgs))]

    def analyzeImages(self, images, fd_option=None):
        """analyzeImage over a batch of frames: detection and all faces as GPU batches; a list of
        Face lists, one per frame."""
        imgs, cim = _image_array(images)
        opt = _det_opt(fd_option or self.options.fd_option)
        cap = 64 * max(1, len(imgs))
        for _ in range(2):
            out = (_Face * cap)()
            owner = np.zeros(cap, np.int32)
            n = ctypes.c_int32()
            _check(lib().ffd_analyze_images(self._h, cim, len(imgs), ctypes.byref(opt), out, owner.ctypes.data, cap,
                                            ctypes.byref(n)), self._h)
            if n.value <= cap:
                break
            cap = n.value
        res = [[] for _ in imgs]
        for i in range(n.value):
            res[owner[i]].append(_face_from_record(out[i]))
        return res

    def detect_device(self, d_images, image_bytes, width, height, stride, n_img, fd_option=None, cap=None):
        """detectFace over n_img frames already in device memory (one size, image_bytes apart):
        (boxes (n, 4) int32, frame index per box (n,) int32), frames in order."""
        opt = _det_opt(fd_option or self.options.fd_option)
        cap = cap or 64 * max(1, n_img)
        for _ in range(2):
            boxes = np.zeros((cap, 4), np.int32)
            owner = np.zeros(cap, np.int32)
            n = ctypes.c_int32()
            _check(lib().ffd_detect_faces_device(self._h, d_images, image_bytes, width, height, stride, n_img,
                                                 ctypes.byref(opt), boxes.ctypes.data, owner.ctypes.data, cap,
                                                 ctypes.byref(n)), self._h)
            if n.value <= cap:
                break
            cap = n.value
        return boxes[: n.value], owner[: n.value]

    def detect_candidates(self, img, fd_option=None):
        """Test hook: detectMultiScale's ungrouped candidates of one frame in scan order, (n, 4)."""
        imgs, cim = _image_array([img])
        opt = _det_opt(fd_option or self.options.fd_option)
        cap = 4096
        for _ in range(2):
            raw = np.zeros((cap, 4), np.int32)
            n = ctypes.c_int32()
            _check(lib().ffd_detect_candidates(self._h, cim, ctypes.byref(opt), raw.ctypes.data, cap,
                                               ctypes.byref(n)), self._h)
            if n.value <= cap:
                break
            cap = n.value
        return raw[: n.value].copy()

    # ---- batched API --------------------------------------------------------
    def analyzeFaces(self, images, boxes, box_img=None):
        n = len(boxes)
        if n == 0:
            return []
        imgs, cim = _image_array(images)
        crect = (_Rect * n)(*[_Rect(*[int(v) for v in b]) for b in boxes])
        cmap = None
        if box_img is not None:
            cmap = np.ascontiguousarray(box_img, np.int32)
        out = (_Face * n)()
        _check(lib().ffd_analyze_faces(self._h, cim, len(imgs), crect,
                                       cmap.ctypes.data if cmap is not None else None, n, out), self._h)
        return [_face_from_record(r) for r in out]

    def analyze_device(self, d_images, image_bytes, width, height, stride, n_img, boxes, box_img, d_out):
        """Enqueue a batch whose images (and output records) live in device memory.  boxes: (n, 4)
        int32 array (x, y, w, h; ffd_rect layout, passed without copying when already packed) or a
        sequence of 4-tuples; box_img: (n,) int32 image index per box, or None."""
        rects = _packed_rects(boxes)
        cmap = np.ascontiguousarray(box_img, np.int32) if box_img is not None else None
        _check(lib().ffd_analyze_faces_device(self._h, d_images, image_bytes, width, height, stride, n_img,
                                              rects.ctypes.data, cmap.ctypes.data if cmap is not None else None,
                                              rects.shape[0], d_out), self._h)
        self._keep = (rects, cmap)

    def synchronize(self):
        _check(lib().ffd_synchronize(self._h), self._h)

    def stream(self):
        return lib().ffd_stream(self._h)

    def check_mag_sqrt(self):
        """ffd_check_mag_sqrt: (floats checked, mismatches) of the Gabor magnitude sqrt vs sqrtf."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().ffd_check_mag_sqrt(self._h, ctypes.byref(a), ctypes.byref(b)), self._h)
        return a.value, b.value

    def set_profiling(self, enable=True):
        _check(lib().ffd_set_profiling(self._h, 1 if enable else 0), self._h)

    def stage_times(self):
        """{stage name: (total device ms, launches)} since set_profiling(True)."""
        ms = np.zeros(NUM_STAGES, np.float64)
        n = np.zeros(NUM_STAGES, np.int64)
        _check(lib().ffd_get_stage_times(self._h, ms.ctypes.data, n.ctypes.data, NUM_STAGES), self._h)
        return {lib().ffd_stage_name(i).decode(): (float(ms[i]), int(n[i])) for i in range(NUM_STAGES)}

    def geometry(self, box_w, box_h):
        v = [ctypes.c_int32() for _ in range(4)]
        _check(lib().ffd_face_geometry(self._h, box_w, box_h, *[ctypes.byref(x) for x in v]), self._h)
        return tuple(x.value for x in v)  # face_w, face_h, n_hp_patches, n_mp_patches

    def extract_channels(self, gray_face):
        """ImageSample(img, {0,1,2}, true).m_feature_channels as 38 x (h+1) x (w+1) uint32."""
        g = np.ascontiguousarray(gray_face, np.uint8)
        h, w = g.shape
        out = np.zeros((NUM_CHANNELS, h + 1, w + 1), np.uint32)
        _check(lib().ffd_extract_channels(self._h, g.ctypes.data, w, h, out.ctypes.data), self._h)
        return out

    def estimateHeadPose(self, channels, face_bbox=None, options=None):
        """FaceForest::estimateHeadPose (src/FaceForest.cpp:60-72) on an image sample's 38 integral
        channels (extract_channels layout); face_bbox = the patch region (default: whole sample);
        options: a HeadPoseEstimatorOption (default: the engine's).  Returns (headpose, variance)."""
        ch = np.ascontiguousarray(channels, np.uint32)
        _, h1, w1 = ch.shape
        r = _Rect(*[int(v) for v in (face_bbox or (0, 0, w1 - 1, h1 - 1))])
        o = None
        if options is not None:
            o = _HpOpt(options.num_head_pose_labels, options.step_size, options.min_foreground_probability)
        hp, var = ctypes.c_float(), ctypes.c_float()
        _check(lib().ffd_estimate_headpose(self._h, ch.ctypes.data, w1 - 1, h1 - 1, ctypes.byref(r),
                                           ctypes.byref(o) if o is not None else None, ctypes.byref(hp),
                                           ctypes.byref(var)), self._h)
        return hp.value, var.value

    def estimateFacialFeatures(self, channels, face_bbox, tree_ids, options=None):
        """FaceForest::estimateFacialFeatures (src/FaceForest.cpp:74-95): the FFD forest made of the
        global tree ids (forest * 20 + tree), options: a MultiPartEstimatorOption (default: the
        engine's), default MeanShiftOption; 10 x 2 int landmarks in sample coordinates ((0, 0) past
        num_parts)."""
        ch = np.ascontiguousarray(channels, np.uint32)
        _, h1, w1 = ch.shape
        r = _Rect(*[int(v) for v in (face_bbox or (0, 0, w1 - 1, h1 - 1))])
        t = np.ascontiguousarray(tree_ids, np.int32)
        o = None
        if options is not None:
            o = _MpOpt(options.num_parts, options.step_size, options.min_samples, options.min_forground,
                       options.min_pf, options.max_variance, options.step_size_y)
        pts = np.zeros((10, 2), np.int32)
        _check(lib().ffd_estimate_facial_features(self._h, ch.ctypes.data, w1 - 1, h1 - 1, ctypes.byref(r),
                                                  t.ctypes.data, t.size, ctypes.byref(o) if o is not None else None,
                                                  pts.ctypes.data), self._h)
        return pts

    def leaves(self, kind, leaf_ids):
        """Leaf payloads (HeadPoseLeaf / MPLeaf members as a dict of arrays) of model leaf ordinals
        (ffd_forest_leaves), what Forest<S>::evaluateMT's Leaf* gives the reference's callers."""
        ids = np.ascontiguousarray(leaf_ids, np.int32).reshape(-1)
        T = _HpLeaf if kind == FOREST_HEADPOSE else _MpLeaf
        out = (T * max(1, ids.size))()
        _check(lib().ffd_forest_leaves(self._h, kind, ids.ctypes.data, ids.size, out), self._h)
        recs = out[: ids.size]
        if kind == FOREST_HEADPOSE:
            return dict(hp_nsamples=np.array([r.hp_nsamples for r in recs], np.int32),
                        hp_foreground=np.array([r.hp_foreground for r in recs], np.float32),
                        hp_labels=np.array([list(r.hp_labels) for r in recs], np.int32).reshape(-1, 5))
        return dict(mp_samples=np.array([r.mp_samples for r in recs], np.int32),
                    mp_foreground=np.array([r.mp_foreground for r in recs], np.float32),
                    mp_parts_offset=np.array([[list(p) for p in r.mp_parts_offset] for r in recs], np.int32).reshape(-1, 10, 2),
                    mp_parts_variance=np.array([list(r.mp_parts_variance) for r in recs], np.float32).reshape(-1, 10),
                    mp_prob_foreground=np.array([list(r.mp_prob_foreground) for r in recs], np.float32).reshape(-1, 10))

    def join(self, comm_id, n_ranks, rank):
        """Join the RCCL communicator `comm_id` (bytes from comm_id() on one rank) as `rank`."""
        buf = (ctypes.c_uint8 * COMM_ID_BYTES).from_buffer_copy(bytes(comm_id))
        _check(lib().ffd_engine_join(self._h, buf, n_ranks, rank), self._h)

    def comm_info(self):
        """(ranks, this rank) of the RCCL communicator the engine joined (ncclCommCount / ncclCommUserRank)."""
        n, r = ctypes.c_int32(), ctypes.c_int32()
        _check(lib().ffd_engine_comm_info(self._h, ctypes.byref(n), ctypes.byref(r)), self._h)
        return n.value, r.value

    def gather(self, d_local, n_per_rank, d_root, root=0):
        """Enqueue the RCCL gather of n_per_rank ffd_face records per rank into d_root on `root`."""
        _check(lib().ffd_gather_faces(self._h, d_local, n_per_rank, d_root, root), self._h)

    def trace(self, index, box_w, box_h):
        """Per-stage intermediates of face `index` of the last batch."""
        fw, fh, nhp, nmp = self.geometry(box_w, box_h)
        bufs = dict(face=np.zeros((fh, fw), np.uint8), channels=np.zeros((NUM_CHANNELS, fh + 1, fw + 1), np.uint32),
                    hp_leaves=np.zeros((nhp, 15), np.int32), mp_leaves=np.zeros(nmp * MAX_TREES, np.int32),
                    trees=np.zeros(MAX_TREES, np.int32), pose_freq=np.zeros(5, np.float32),
                    vote_counts=np.zeros(10, np.int32), ms_mean=np.zeros((10, 2), np.float32))
        tr = _Trace(*[bufs[k].ctypes.data for k, _ in _Trace._fields_])
        _check(lib().ffd_get_trace(self._h, index, ctypes.byref(tr)), self._h)
        nt = int((bufs["trees"] >= 0).sum())
        bufs["trees"] = bufs["trees"][:nt]
        bufs["mp_leaves"] = bufs["mp_leaves"][: nmp * nt].reshape(nmp, nt)
        return bufs


class _ForestParamC(ctypes.Structure):  # ffd_forest_param = ForestParam (Constants.hpp:24-60)
    _fields_ = [("max_depth", ctypes.c_int32), ("min_patches", ctypes.c_int32), ("ntests", ctypes.c_int32),
                ("ntrees", ctypes.c_int32), ("nimages", ctypes.c_int32), ("npatches", ctypes.c_int32),
                ("face_size", ctypes.c_int32), ("patch_size_ratio", ctypes.c_float), ("tree_path", ctypes.c_char_p),
                ("image_path", ctypes.c_char_p), ("features", ctypes.POINTER(ctypes.c_int32)),
                ("n_features", ctypes.c_int32)]


def convert_model(hp_config, ffd_config, cascade_xml, out_path):
    """FaceForest(FaceForestOptions)'s loads (src/FaceForest.cpp:15-58) as a model file: loadConfigFile of both
    configs, the head-pose trees of hp tree_path, the FFD trees of the sorted sub-directories of the FFD
    tree_path, the Haar cascade (ffd_model_convert).  Returns out_path."""
    from . import config
    keep = []

    def c_param(path):
        ok, p = config.load_config_file(path)
        if not ok:
            raise FFDError(0, f"cannot read {path}")
        feats = (ctypes.c_int32 * max(1, len(p.features)))(*p.features)
        keep.append(feats)
        return _ForestParamC(p.max_depth, p.min_patches, p.ntests, p.ntrees, p.nimages, p.npatches, p.face_size,
                             p.patch_size_ratio, p.tree_path.encode(), p.image_path.encode(), feats, len(p.features))

    hp, mp = c_param(hp_config), c_param(ffd_config)
    root = mp.tree_path.decode()
    dirs = sorted(os.path.join(root, d) for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
    arr = (ctypes.c_char_p * max(1, len(dirs)))(*[d.encode() for d in dirs])
    st = lib().ffd_model_convert(ctypes.byref(hp), ctypes.byref(mp), arr, len(dirs),
                                 cascade_xml.encode() if cascade_xml else None, str(out_path).encode())
    if st != 0:
        raise FFDError(st, "ffd_model_convert: " + lib().ffd_model_convert_last_error().decode())
    return out_path


def comm_id():
    """ncclGetUniqueId through libffd (FFD_COMM_ID_BYTES bytes, to be shared with the other ranks)."""
    buf = (ctypes.c_uint8 * COMM_ID_BYTES)()
    st = lib().ffd_comm_id(buf)
    if st != 0:
        raise FFDError(st, lib().ffd_group_last_error(None).decode(errors="replace"))
    return bytes(buf)


class FaceForestGroup:
    """One process driving several devices (ffd_group_*): faces sharded in contiguous blocks,
    one engine (model copy) per device, one RCCL gather of the records."""

    def __init__(self, devices, options=None):
        self.options = options or FaceForestOptions()
        d, self._path = _make_desc(self.options)
        devs = (ctypes.c_int32 * len(devices))(*devices)
        h = ctypes.c_void_p()
        st = lib().ffd_group_create(ctypes.byref(d), devs, len(devices), ctypes.byref(h))
        if st != 0:
            raise FFDError(st, lib().ffd_group_last_error(None).decode(errors="replace"))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().ffd_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def size(self):
        return lib().ffd_group_size(self._h)

    def analyzeFaces(self, images, boxes, box_img=None):
        n = len(boxes)
        if n == 0:
            return []
        imgs, cim = _image_array(images)
        rects = _packed_rects(boxes)
        cmap = np.ascontiguousarray(box_img, np.int32) if box_img is not None else None
        out = (_Face * n)()
        st = lib().ffd_group_analyze_faces(self._h, cim, len(imgs), rects.ctypes.data,
                                           cmap.ctypes.data if cmap is not None else None, n, out)
        if st != 0:
            raise FFDError(st, lib().ffd_group_last_error(self._h).decode(errors="replace"))
        return [_face_from_record(r) for r in out]


class ImageSample:
    """ImageSample (src/ImageSample.cpp:11-20, include/ImageSample.hpp:146-190) kept in HBM (ffd_sample_create):
    the 38 integral channels of an 8-bit gray face, with Forest<S>::evaluateMT on its patches (a list or the
    estimators' grid) and the static estimators of FaceForest on it.  Owned by the FaceForest that made it;
    close() (or a with-block) frees it."""

    def __init__(self, face_forest, gray=None, channels=None):
        self.ff = face_forest
        h = ctypes.c_void_p()
        if channels is not None:
            ch = np.ascontiguousarray(channels, np.uint32)
            _check(lib().ffd_sample_create_from_channels(face_forest.handle, ch.ctypes.data, ch.shape[2] - 1,
                                                         ch.shape[1] - 1, ctypes.byref(h)), face_forest.handle)
        else:
            g = np.ascontiguousarray(gray, np.uint8)
            if g.ndim != 2:
                raise ValueError("ImageSample: an 8-bit single-channel (gray) face")
            _check(lib().ffd_sample_create(face_forest.handle, g.ctypes.data, g.shape[1], g.shape[0], g.strides[0],
                                           ctypes.byref(h)), face_forest.handle)
        self._h = h.value
        w, hh = ctypes.c_int32(), ctypes.c_int32()
        lib().ffd_sample_size(self._h, ctypes.byref(w), ctypes.byref(hh))
        self.width, self.height = w.value, hh.value

    def close(self):
        if getattr(self, "_h", None):
            lib().ffd_sample_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def channels(self):
        out = np.zeros((38, self.height + 1, self.width + 1), np.uint32)
        _check(lib().ffd_sample_channels(self._h, out.ctypes.data), self.ff.handle)
        return out

    def eval_leaves(self, kind, patches_xy, tree_ids):
        p = np.ascontiguousarray(patches_xy, np.int32).reshape(-1, 2)
        t = np.ascontiguousarray(tree_ids, np.int32)
        out = np.zeros((p.shape[0], t.size), np.int32)
        _check(lib().ffd_sample_eval_leaves(self._h, kind, p.ctypes.data, p.shape[0], t.ctypes.data, t.size,
                                            out.ctypes.data), self.ff.handle)
        return out

    def eval_grid(self, kind, x0, y0, step, nx, ny, tree_ids):
        t = np.ascontiguousarray(tree_ids, np.int32)
        out = np.zeros((nx * ny, t.size), np.int32)
        _check(lib().ffd_sample_eval_grid(self._h, kind, x0, y0, step, nx, ny, t.ctypes.data, t.size, out.ctypes.data),
               self.ff.handle)
        return out

    def estimateHeadPose(self, face_bbox=None, options=None):
        r = _Rect(*face_bbox) if face_bbox is not None else None
        o = None
        if options is not None:
            o = _HpOpt(options.num_head_pose_labels, options.step_size, options.min_foreground_probability)
        hp, var = ctypes.c_float(), ctypes.c_float()
        _check(lib().ffd_sample_estimate_headpose(self._h, ctypes.byref(r) if r else None, ctypes.byref(o) if o else None,
                                                  ctypes.byref(hp), ctypes.byref(var)), self.ff.handle)
        return hp.value, var.value

    def estimateFacialFeatures(self, face_bbox, tree_ids, options=None):
        r = _Rect(*face_bbox) if face_bbox is not None else None
        t = np.ascontiguousarray(tree_ids, np.int32)
        o = None
        if options is not None:
            o = _MpOpt(options.num_parts, options.step_size, options.min_samples, options.min_forground,
                       options.min_pf, options.max_variance, getattr(options, "step_size_y", 0))
        pts = np.zeros((10, 2), np.int32)
        _check(lib().ffd_sample_estimate_facial_features(self._h, ctypes.byref(r) if r else None, t.ctypes.data, t.size,
                                                         ctypes.byref(o) if o else None, pts.ctypes.data), self.ff.handle)
        return pts


def meanshift(face_forest, votes, option=None):
    """MeanShift::shift (include/MeanShift.hpp:41-76) of one vote list on the GPU: votes = [(x, y, weight, check)];
    returns the mode before rounding (the reference's Point_<int> result is its cvRound)."""
    v = np.zeros(len(votes), dtype=[("x", "<i4"), ("y", "<i4"), ("w", "<f4"), ("c", "<i4")])
    for i, (x, y, w, c) in enumerate(votes):
        v[i] = (x, y, w, int(bool(c)))
    o = option or MeanShiftOption()
    mo = _MsOpt(o.kernel_size, o.max_iterations, o.stopping_criteria)
    out = np.zeros(2, np.float32)
    _check(lib().ffd_meanshift(face_forest.handle, v.ctypes.data if len(v) else None, len(v), ctypes.byref(mo),
                               out.ctypes.data), face_forest.handle)
    return out


class Forest:
    """Forest<S>::evaluateMT over a batch of patches (include/Forest.hpp:80-90)."""

    def __init__(self, face_forest, kind):
        self.ff = face_forest
        self.kind = kind

    def evaluate(self, channels, patches_xy, tree_ids):
        ch = np.ascontiguousarray(channels, np.uint32)
        _, h1, w1 = ch.shape
        p = np.ascontiguousarray(patches_xy, np.int32).reshape(-1, 2)
        t = np.ascontiguousarray(tree_ids, np.int32)
        out = np.zeros((p.shape[0], t.size), np.int32)
        _check(lib().ffd_forest_eval_leaves(self.ff.handle, self.kind, ch.ctypes.data, w1 - 1, h1 - 1, p.ctypes.data,
                                            p.shape[0], t.ctypes.data, t.size, out.ctypes.data), self.ff.handle)
        return out
