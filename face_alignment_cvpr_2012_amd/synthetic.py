"""Synthetic workloads of BASELINE.json's configs, seeded and deterministic.

C2: crop k = bundled fixture face (k mod 20), annotated bbox jittered by dx, dy ~ U{-6..6} and
scale ~ U[0.95, 1.05], resampled (bilinear, edge-clamped) to 150x150, plus N(0, 2^2) pixel
noise clipped to [0, 255]; seed 2012.  analyzeFace(crop, Rect(0, 0, 150, 150)) then scales the
crop to a 125x125 face (576 head-pose + 1,024 FFD patches).

C3: 1920x1080 frames; background = seeded smooth noise (bilinear upsampling of a coarse random
grid); 8 fixture faces per frame pasted at random non-overlapping positions with face-box sides
U{100..200} px.  The analysis boxes are the paste boxes put through the reference's detectFace
enlargement (face_box_from_detection, src/FaceForest.cpp:148-158), so the scaled faces are
125 x ~148 like Haar boxes.

C5: C2-style crops, 64 per frame x 512 frames = 32,768 faces.
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = os.path.join(os.path.dirname(HERE), "tests", "golden", "faces.npz")


def load_fixtures(path=FIXTURES):
    d = np.load(path, allow_pickle=False)
    return {k: d[k] for k in d.files}


def _bilinear(img, xs, ys):
    """Sample HxWx3 uint8 img at float coords (edge clamped); xs: (S,), ys: (S,) grids."""
    h, w = img.shape[:2]
    x0 = np.clip(np.floor(xs).astype(np.int64), 0, w - 1)
    y0 = np.clip(np.floor(ys).astype(np.int64), 0, h - 1)
    x1 = np.clip(x0 + 1, 0, w - 1)
    y1 = np.clip(y0 + 1, 0, h - 1)
    fx = np.clip(xs - np.floor(xs), 0, 1)[None, :, None]
    fy = np.clip(ys - np.floor(ys), 0, 1)[:, None, None]
    f = img.astype(np.float32)
    a = f[y0][:, x0] * (1 - fx) + f[y0][:, x1] * fx
    b = f[y1][:, x0] * (1 - fx) + f[y1][:, x1] * fx
    return a * (1 - fy) + b * fy


def make_crops(n, size=150, seed=2012, fixtures=None):
    """Return (crops uint8 [n, size, size, 3] BGR, source fixture index [n])."""
    fx = fixtures or load_fixtures()
    imgs, boxes = fx["images"], fx["boxes"]
    rng = np.random.default_rng(seed)
    out = np.empty((n, size, size, 3), np.uint8)
    src = np.arange(n) % len(imgs)
    jit = rng.integers(-6, 7, size=(n, 2))
    scl = rng.uniform(0.95, 1.05, size=n)
    for k in range(n):
        i = src[k]
        x, y, w, h = boxes[i]
        cx = x + w / 2.0 + jit[k, 0]
        cy = y + h / 2.0 + jit[k, 1]
        side = w * scl[k]
        t = (np.arange(size) + 0.5) / size
        xs = cx - side / 2.0 + t * side - 0.5
        ys = cy - side / 2.0 + t * side - 0.5
        v = _bilinear(imgs[i], xs, ys)
        v += rng.normal(0.0, 2.0, size=v.shape).astype(np.float32)
        out[k] = np.clip(np.rint(v), 0, 255).astype(np.uint8)
    return out, src


def crop_ground_truth(n, size=150, seed=2012, fixtures=None):
    """The annotated landmarks (data/imgs/index_random_subset.txt, faces.npz 'parts', box-relative) of the n
    crops make_crops(n, size, seed) returns, mapped into crop pixel coordinates, float64 [n, 10, 2].
    analyzeFace(crop, Rect(0, 0, size, size)) reports bbox-relative points, i.e. the same frame.
    The jitter / scale draws are the first two of make_crops' generator, so they are re-drawn here."""
    fx = fixtures or load_fixtures()
    boxes, parts = fx["boxes"], fx["parts"].astype(np.float64)
    rng = np.random.default_rng(seed)
    src = np.arange(n) % len(boxes)
    jit = rng.integers(-6, 7, size=(n, 2))
    scl = rng.uniform(0.95, 1.05, size=n)
    x, y, w, h = (boxes[src, j].astype(np.float64) for j in range(4))
    cx = x + w / 2.0 + jit[:, 0]
    cy = y + h / 2.0 + jit[:, 1]
    side = w * scl
    # make_crops samples crop pixel u at source coordinate cx - side/2 + (u + 0.5) side/size - 0.5
    gt = np.empty((n, parts.shape[1], 2), np.float64)
    gt[:, :, 0] = (parts[src, :, 0] + x[:, None] + 0.5 - (cx - side / 2.0)[:, None]) * (size / side)[:, None] - 0.5
    gt[:, :, 1] = (parts[src, :, 1] + y[:, None] + 0.5 - (cy - side / 2.0)[:, None]) * (size / side)[:, None] - 0.5
    return gt


def _interp_matrix(n, m, cell=64.0):
    """(n, m) matrix of linear interpolation weights: output i samples coarse coordinate
    (i + 0.5) / cell (edge clamped), as _bilinear does along one axis."""
    t = (np.arange(n) + 0.5) / cell
    i0 = np.clip(np.floor(t).astype(np.int64), 0, m - 1)
    i1 = np.clip(i0 + 1, 0, m - 1)
    f = np.clip(t - np.floor(t), 0, 1).astype(np.float32)
    M = np.zeros((n, m), np.float32)
    M[np.arange(n), i0] += 1 - f
    M[np.arange(n), i1] += f
    return M


def face_box_from_detection(det, img_w, img_h):
    """detectFace's widening of a (Haar) detection, src/FaceForest.cpp:148-158: 5 % of the width
    on each side, height + 2 x 15 % of the width (below the box), clipped to the image by
    intersect (src/face_utils.cpp:325-346)."""
    x, y, w, h = (int(v) for v in det)
    ox, oy = int(w * 0.05), int(w * 0.15)
    r = (x - ox, y, w + 2 * ox, h + 2 * oy)
    ix, iy = max(r[0], 0), max(r[1], 0)
    iw = min(r[0] + r[2], img_w) - ix
    ih = min(r[1] + r[3], img_h) - iy
    if iw <= 0 or ih <= 0:
        return (0, 0, 0, 0)
    return (ix, iy, iw, ih)


def make_frames(n_frames, faces_per_frame=8, width=1920, height=1080, seed=1080, fixtures=None):
    """Return (frames uint8 [n, height, width, 3] BGR, boxes int32 [n, faces_per_frame, 4] analysis
    boxes (detectFace-enlarged), paste boxes int32 [n, faces_per_frame, 4])."""
    fx = fixtures or load_fixtures()
    imgs, fboxes = fx["images"], fx["boxes"]
    rng = np.random.default_rng(seed)
    frames = np.empty((n_frames, height, width, 3), np.uint8)
    boxes = np.zeros((n_frames, faces_per_frame, 4), np.int32)
    paste = np.zeros((n_frames, faces_per_frame, 4), np.int32)
    gy, gx = (height + 63) // 64 + 1, (width + 63) // 64 + 1
    for f in range(n_frames):
        coarse = rng.uniform(40, 200, size=(gy, gx, 3)).astype(np.float32)
        # bilinear upsampling of the coarse grid as two interpolation matrices (separable)
        my, mx = _interp_matrix(height, gy), _interp_matrix(width, gx)
        bg = np.stack([my @ coarse[:, :, c] @ mx.T for c in range(3)], axis=-1)
        frame = np.clip(np.rint(bg), 0, 255).astype(np.uint8)
        taken = []
        for k in range(faces_per_frame):
            i = int(rng.integers(0, len(imgs)))
            side = int(rng.integers(100, 201))
            region = int(round(side * 1.6))  # pasted square around the face box
            for _ in range(1000):
                px = int(rng.integers(0, width - region))
                py = int(rng.integers(0, height - region))
                if all(px + region <= a or a + b <= px or py + region <= c or c + d <= py for a, c, b, d in taken):
                    break
            else:
                raise RuntimeError("could not place a face")
            taken.append((px, py, region, region))
            x, y, w, h = (float(v) for v in fboxes[i])
            scale = side / w
            cx, cy = x + w / 2.0, y + h / 2.0
            t = (np.arange(region) + 0.5) / scale
            src_x = cx - region / (2 * scale) + t - 0.5
            src_y = cy - region / (2 * scale) + t - 0.5
            patch = _bilinear(imgs[i], src_x, src_y)
            frame[py:py + region, px:px + region] = np.clip(np.rint(patch), 0, 255).astype(np.uint8)
            # face box inside the paste: the fixture box scaled; detection = that box
            bx = px + int(round(region / 2.0 - side / 2.0))
            by = py + int(round(region / 2.0 - h * scale / 2.0))
            det = (bx, by, side, int(round(h * scale)))
            paste[f, k] = det
            boxes[f, k] = face_box_from_detection(det, width, height)
        frames[f] = frame
    return frames, boxes, paste


def training_rois(n, face_size=125, seed=7, fixtures=None):
    """Training ROIs for facial-feature tree training, following trainTree
    (src/train_ffd.cpp:82-99): image k = bundled fixture k mod 20 (k >= 20: horizontally jittered,
    rescaled and noised variants, seeded), scaled so the face box is face_size wide (bilinear,
    edge-clamped; not OpenCV's resize, the ROIs are inputs, not parity subjects), then the box
    enlarged by 10 % per side and clipped to the image (face_utils.cpp enlargeFace).  Returns
    (list of uint8 gray ROIs, int32 [n, 10, 2] landmarks in ROI pixels).  The LFW training set the
    reference trains on (config_ffd.txt) is not in the repository."""
    fx = fixtures or load_fixtures()
    imgs, boxes, parts = fx["images"], fx["boxes"], fx["parts"]
    rng = np.random.default_rng(seed)
    rois, pts = [], np.zeros((n, 10, 2), np.int32)
    for k in range(n):
        i = k % len(imgs)
        x, y, w, h = (float(v) for v in boxes[i])
        p = parts[i].astype(np.float64) + np.array([x, y])  # image coordinates
        jit = np.zeros(2) if k < len(imgs) else rng.uniform(-4, 4, size=2)
        scl = 1.0 if k < len(imgs) else rng.uniform(0.93, 1.07)
        s = face_size / (w * scl)
        H, W = imgs[i].shape[:2]
        sw, sh = int(W * s), int(H * s)
        xs = (np.arange(sw) + 0.5) / s - 0.5 + jit[0]
        ys = (np.arange(sh) + 0.5) / s - 0.5 + jit[1]
        bgr = _bilinear(imgs[i], xs, ys)
        gray = (bgr[..., 0] * 0.114 + bgr[..., 1] * 0.587 + bgr[..., 2] * 0.299)
        if k >= len(imgs):
            gray = gray + rng.normal(0.0, 2.0, size=gray.shape)
        gray = np.clip(np.rint(gray), 0, 255).astype(np.uint8)
        bx, by, bw, bh = int((x - jit[0]) * s), int((y - jit[1]) * s), int(w * s), int(h * s)
        ox, oy = int(bw * 0.1), int(bh * 0.1)
        x0, y0 = max(bx - ox, 0), max(by - oy, 0)
        x1, y1 = min(bx - ox + bw + 2 * ox, sw), min(by - oy + bh + 2 * oy, sh)
        rois.append(np.ascontiguousarray(gray[y0:y1, x0:x1]))
        q = (p - jit) * s
        pts[k] = np.rint(q - np.array([x0, y0])).astype(np.int32)
    return rois, pts


def headpose_training_images(n, face_size=125, seed=11, margin=40, fixtures=None):
    """Training images for head-pose tree training, following train_headpose.cpp's
    trainTree (src/train_headpose.cpp:83-96): image k = bundled fixture k mod 20 (k >= 20: jittered,
    rescaled and noised variants, seeded), scaled so the face box is face_size wide (bilinear,
    edge-clamped; not OpenCV's resize: the images are inputs, not parity subjects) and cut to the face
    box plus `margin` pixels on every side (edge-clamped where that leaves the photograph), so that
    every positive patch lies inside the image and the negatives have room around the face.  The
    fixtures carry no head-pose annotation, so the pose label is synthetic: k mod 5 - 2.  Returns (list
    of uint8 gray images, int32 [n, 4] boxes (x, y, w, h) in them, int32 [n] poses)."""
    fx = fixtures or load_fixtures()
    imgs, boxes = fx["images"], fx["boxes"]
    rng = np.random.default_rng(seed)
    out, bx_out, poses = [], np.zeros((n, 4), np.int32), np.zeros(n, np.int32)
    for k in range(n):
        i = k % len(imgs)
        x, y, w, h = (float(v) for v in boxes[i])
        jit = np.zeros(2) if k < len(imgs) else rng.uniform(-4, 4, size=2)
        scl = 1.0 if k < len(imgs) else rng.uniform(0.93, 1.07)
        s = face_size / (w * scl)
        bx, by, bw, bh = int(x * s), int(y * s), int(w * s), int(h * s)
        ow, oh = max(bw, face_size) + 2 * margin, max(bh, face_size) + 2 * margin
        xs = (np.arange(bx - margin, bx - margin + ow) + 0.5) / s - 0.5 + jit[0]
        ys = (np.arange(by - margin, by - margin + oh) + 0.5) / s - 0.5 + jit[1]
        bgr = _bilinear(imgs[i], xs, ys)
        gray = (bgr[..., 0] * 0.114 + bgr[..., 1] * 0.587 + bgr[..., 2] * 0.299)
        if k >= len(imgs):
            gray = gray + rng.normal(0.0, 2.0, size=gray.shape)
        out.append(np.clip(np.rint(gray), 0, 255).astype(np.uint8))
        bx_out[k] = (margin, margin, bw, bh)
        poses[k] = k % 5 - 2
    return out, bx_out, poses
