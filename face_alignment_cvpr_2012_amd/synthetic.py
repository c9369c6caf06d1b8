"""Synthetic workloads of BASELINE.json's configs, seeded and deterministic.

C2: crop k = bundled fixture face (k mod 20), annotated bbox jittered by dx, dy ~ U{-6..6} and
scale ~ U[0.95, 1.05], resampled (bilinear, edge-clamped) to 150x150, plus N(0, 2^2) pixel
noise clipped to [0, 255]; seed 2012.  analyzeFace(crop, Rect(0, 0, 150, 150)) then scales the
crop to a 125x125 face (576 head-pose + 1,024 FFD patches).
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
