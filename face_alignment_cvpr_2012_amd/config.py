"""Harness-side IO of the reference: configuration files, annotations, images.

Mirrors src/face_utils.cpp:18-181 and include/Constants.hpp:24-68:

* ``ForestParam`` / ``load_config_file`` — Constants.hpp:24-60 and loadConfigFile (face_utils.cpp:50-140):
  the positional text config (a caption line before every value), with the reference's defaults when
  the file is missing.
* ``FaceAnnotation`` / ``load_annotations`` — face_utils.hpp:23-29 and loadAnnotations
  (face_utils.cpp:143-181): ``url x y w h pose n x0 y0 ... x(n-1) y(n-1)`` per line, fields split on
  single spaces (boost::is_any_of(" ")), ``#`` lines skipped.
* ``load_image`` — loadImage (face_utils.cpp:18-28): the image named by an annotation, looked up in the
  directory of the annotation file's path.  OpenCV is not in this image, so decoding is pluggable
  (``ImageStore``): pre-decoded BGR arrays (an ``.npz`` of name -> array, or ``<name>.npy`` files), or
  Pillow for JPEG/PNG (its IDCT may round differently from cv::imread's libjpeg — decoded pixels are
  inputs, not a parity claim).
* ``intersect`` / ``enlarge_face`` — face_utils.cpp:325-346 and :30-48.
* ``split_by_pose`` — eval_ffd's split (src/eval_ffd.cpp:153-169): annotations bucketed by pose + 2
  into NUM_HEADPOSE_CLASSES, the first int(size * 0.9f) of each bucket train, the rest test.
"""
import os
from dataclasses import dataclass, field

import numpy as np

TRAIN_IMAGES_PERCENTAGE = np.float32(0.9)  # Constants.hpp:65
NUM_HEADPOSE_CLASSES = 5                    # Constants.hpp:66


@dataclass
class ForestParam:                          # include/Constants.hpp:24-60 (the defaults of loadConfigFile's failure path)
    max_depth: int = 15
    min_patches: int = 20
    ntests: int = 250
    ntrees: int = 10
    nimages: int = 500
    npatches: int = 200
    face_size: int = 100
    patch_size_ratio: float = 0.25
    tree_path: str = ""
    image_path: str = ""
    features: list = field(default_factory=list)

    def getPatchSize(self):                 # Constants.hpp:26-30: round(face_size * patch_size_ratio)
        return int(np.round(np.float32(self.face_size) * np.float32(self.patch_size_ratio)))


def load_config_file(path):
    """loadConfigFile (face_utils.cpp:50-140): returns (ok, ForestParam).  A missing file gives the
    reference's defaults and ok = False; a malformed value raises ValueError (boost::lexical_cast throws)."""
    p = ForestParam()
    if not os.path.exists(path):
        return False, p
    with open(path) as f:
        lines = f.read().split("\n")
    vals = lines[1::2]  # every value follows its caption line

    def at(i):
        if i >= len(vals):
            raise ValueError(f"{path}: missing value {i}")
        return vals[i]
    p.image_path = at(0)
    p.tree_path = at(1)
    p.ntrees = int(at(2))
    p.ntests = int(at(3))
    p.max_depth = int(at(4))
    p.min_patches = int(at(5))
    p.nimages = int(at(6))
    p.npatches = int(at(7))
    p.face_size = int(at(8))
    p.patch_size_ratio = float(np.float32(float(at(9))))
    p.features = [int(float(s)) for s in at(10).split(" ")]  # lexical_cast<float> pushed into vector<int>
    return True, p


@dataclass
class FaceAnnotation:                       # include/face_utils.hpp:23-29
    url: str
    bbox: tuple                             # x, y, width, height
    pose: int
    parts: np.ndarray                       # n x 2 int


def _lexical_int(s):
    if not s or s.strip() != s:
        raise ValueError(f"bad integer field {s!r}")
    return int(s)


def parse_annotations(text):
    """loadAnnotations' line grammar (face_utils.cpp:155-177)."""
    anns = []
    lines = text.split("\n")
    if lines and lines[-1] == "":
        lines.pop()  # std::getline yields no line after the final newline
    for line in lines:
        s = line.split(" ")
        if s[0] == "#":
            continue
        bbox = tuple(_lexical_int(v) for v in s[1:5])
        pose = _lexical_int(s[5])
        n = _lexical_int(s[6])
        parts = np.array([[_lexical_int(s[7 + 2 * i]), _lexical_int(s[8 + 2 * i])] for i in range(n)], np.int32)
        anns.append(FaceAnnotation(s[0], bbox, pose, parts.reshape(n, 2)))
    return anns


def load_annotations(path):
    """loadAnnotations (face_utils.cpp:143-181): returns (ok, [FaceAnnotation])."""
    if not os.path.exists(path):
        return False, []
    with open(path) as f:
        return True, parse_annotations(f.read())


def image_dir(path):
    """loadImage's directory: path up to and including its last '/' (face_utils.cpp:25-26)."""
    return path[:path.rfind("/") + 1]


class ImageStore:
    """loadImage (face_utils.cpp:18-28) without OpenCV: BGR uint8 arrays by image name.

    Sources, first match wins: `arrays` (a dict or an .npz path of name -> HxWx3 BGR), then
    `<dir>/<name>.npy`, then `<dir>/<name>` decoded by Pillow (RGB -> BGR, as cv::IMREAD_COLOR).
    A name found nowhere gives None (the reference's empty Mat: evalForest skips the face)."""

    def __init__(self, directory="", arrays=None):
        self.dir = directory
        if isinstance(arrays, (str, os.PathLike)):
            z = np.load(arrays, allow_pickle=False)
            if "names" in z.files and "images" in z.files:
                arrays = {str(n): im for n, im in zip(z["names"], z["images"])}
            else:
                arrays = {k: z[k] for k in z.files}
        self.arrays = arrays or {}

    def __call__(self, name):
        if name in self.arrays:
            return np.ascontiguousarray(self.arrays[name], np.uint8)
        p = self.dir + name
        if os.path.exists(p + ".npy"):
            return np.ascontiguousarray(np.load(p + ".npy", allow_pickle=False), np.uint8)
        if os.path.exists(p):
            try:
                from PIL import Image
            except ImportError:
                return None
            try:
                rgb = np.asarray(Image.open(p).convert("RGB"))
            except OSError:
                return None
            return np.ascontiguousarray(rgb[:, :, ::-1])
        return None


def intersect(r1, r2):
    """face_utils.cpp:325-346 (x, y, w, h rectangles)."""
    x = r2[0] if r1[0] < r2[0] else r1[0]
    y = r2[1] if r1[1] < r2[1] else r1[1]
    w = (r1[0] + r1[2] if r1[0] + r1[2] < r2[0] + r2[2] else r2[0] + r2[2]) - x
    h = (r1[1] + r1[3] if r1[1] + r1[3] < r2[1] + r2[3] else r2[1] + r2[3]) - y
    if w <= 0 or h <= 0:
        return (0, 0, 0, 0)
    return (x, y, w, h)


def enlarge_face(img_shape, annotation):
    """enlargeFace (face_utils.cpp:30-48): the box grown by 10 % of its size on every side and clipped to
    the image; returns (enlarged box, annotation in the enlarged box's frame: bbox (0, 0, w, h), parts
    shifted by the offset)."""
    bx, by, bw, bh = annotation.bbox
    ox, oy = int(bw * 0.1), int(bh * 0.1)  # cv::Point2i(double, double): truncation
    aux = (bx - ox, by - oy, bw + 2 * ox, bh + 2 * oy)
    e = intersect(aux, (0, 0, int(img_shape[1]), int(img_shape[0])))
    ann = FaceAnnotation(annotation.url, (0, 0, e[2], e[3]), annotation.pose,
                         np.asarray(annotation.parts, np.int32) + np.array([ox, oy], np.int32))
    return e, ann


def split_by_pose(annotations):
    """eval_ffd main (src/eval_ffd.cpp:153-169): (train, test), each a list of NUM_HEADPOSE_CLASSES buckets in
    file order; a bucket's first int(size * 0.9f) annotations train, the rest test."""
    buckets = [[] for _ in range(NUM_HEADPOSE_CLASSES)]
    for a in annotations:
        if not 0 <= a.pose + 2 < NUM_HEADPOSE_CLASSES:  # ann[pose + 2] is out of bounds in the reference
            raise IndexError(f"{a.url}: pose {a.pose} outside [-2, 2]")
        buckets[a.pose + 2].append(a)
    train, test = [], []
    for b in buckets:
        k = int(np.float32(len(b)) * TRAIN_IMAGES_PERCENTAGE)
        train.append(b[:k])
        test.append(b[k:])
    return train, test
