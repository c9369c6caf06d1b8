"""Generate tests/golden/faces.npz from the reference's bundled data (run in the
build container only; the output is committed and is all the GPU box sees).

Inputs (reference, read-only):
  data/imgs/*.jpg                       20 LFW 250x250 faces
  data/imgs/index_random_subset.txt     url, bbox x y w h, pose, 10 landmarks
    (format parsed by loadAnnotations, /root/reference/src/face_utils.cpp:142-181)

The JPEGs are decoded with Pillow (the reference uses cv::imread; OpenCV is not
in this image, so decoded pixels may differ from the reference's by JPEG IDCT
rounding — the fixtures are inputs, not expected outputs).  Channel order is
converted to BGR to match cv::IMREAD_COLOR.
"""
import os
import sys

import numpy as np
from PIL import Image

REF = os.environ.get("FFD_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "faces.npz")


def main():
    idx = os.path.join(REF, "data", "imgs", "index_random_subset.txt")
    names, boxes, poses, parts, imgs = [], [], [], [], []
    with open(idx) as f:
        for line in f:
            s = line.split()
            if not s or s[0] == "#":
                continue
            names.append(s[0])
            boxes.append([int(v) for v in s[1:5]])
            poses.append(int(s[5]))
            n = int(s[6])
            parts.append([[int(s[7 + 2 * i]), int(s[8 + 2 * i])] for i in range(n)])
            rgb = np.asarray(Image.open(os.path.join(REF, "data", "imgs", s[0])).convert("RGB"))
            imgs.append(np.ascontiguousarray(rgb[:, :, ::-1]))
    shapes = {im.shape for im in imgs}
    assert len(shapes) == 1, shapes
    np.savez_compressed(
        OUT,
        names=np.array(names),
        images=np.stack(imgs).astype(np.uint8),
        boxes=np.array(boxes, np.int32),
        poses=np.array(poses, np.int32),
        parts=np.array(parts, np.int32),
    )
    print("wrote", OUT, len(names), "faces", imgs[0].shape)


if __name__ == "__main__":
    sys.exit(main())
