"""Known-answer and invariance tests of the CPU restatement (oracle/), plus the end-to-end
accuracy sanity band against the reference's published errors (output/errors.txt)."""
import numpy as np
import pytest
from scipy.signal import correlate2d

from conftest import crops


def test_bgr2gray_fixed_point(oracle_mod):
    # cvtColor BGR2GRAY 8U: (B*1868 + G*9617 + R*4899 + 8192) >> 14
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0], [10, 200, 30]]], np.uint8)
    g = oracle_mod.bgr2gray(px)
    exp = [(int(b) * 1868 + int(gg) * 9617 + int(r) * 4899 + 8192) >> 14 for b, gg, r in px[0]]
    assert g[0].tolist() == exp == [29, 150, 76, 255, 0, 128]


def test_resize_invariants(oracle_mod):
    rng = np.random.default_rng(1)
    src = rng.integers(0, 256, (150, 150), dtype=np.uint8)
    assert np.array_equal(oracle_mod.resize(src, 150, 150), src)  # equal size: copy
    const = np.full((150, 150), 77, np.uint8)
    assert (oracle_mod.resize(const, 125, 125) == 77).all()
    # exact 2x down-scale: INTER_AREA fast path (a+b+c+d+2)>>2
    s = src[:100, :100].astype(np.int32)
    exp = (s[0::2, 0::2] + s[0::2, 1::2] + s[1::2, 0::2] + s[1::2, 1::2] + 2) >> 2
    assert np.array_equal(oracle_mod.resize(src[:100, :100], 50, 50), exp)
    # bilinear result stays within the local source range
    r = oracle_mod.resize(src, 125, 125)
    assert r.shape == (125, 125) and abs(int(r.mean()) - int(src.mean())) <= 3


def test_channels_known_answers(oracle_mod):
    rng = np.random.default_rng(2)
    face = rng.integers(0, 256, (60, 50), dtype=np.uint8)
    ch = oracle_mod.channels(face)
    assert ch.shape == (38, 61, 51)
    # channel 0 = integral of the gray face
    ii = np.zeros((61, 51), np.int64)
    ii[1:, 1:] = face.astype(np.int64).cumsum(0).cumsum(1)
    assert np.array_equal(ch[0], ii)
    # every channel is an integral image of a u8 plane
    for c in range(38):
        plane = np.diff(np.diff(ch[c].astype(np.int64), axis=0), axis=1)
        assert plane.min() >= 0 and plane.max() <= 255
        assert (ch[c][0] == 0).all() and (ch[c][:, 0] == 0).all()
    # Sobel: reflect-101 borders, saturated to [0,255]; ch36 = d/dy, ch37 = d/dx
    p = np.pad(face.astype(np.int64), 1, mode="reflect")
    dy = (p[2:, :-2] + 2 * p[2:, 1:-1] + p[2:, 2:]) - (p[:-2, :-2] + 2 * p[:-2, 1:-1] + p[:-2, 2:])
    dx = (p[:-2, 2:] + 2 * p[1:-1, 2:] + p[2:, 2:]) - (p[:-2, :-2] + 2 * p[1:-1, :-2] + p[2:, :-2])
    for c, d in ((36, dy), (37, dx)):
        plane = np.diff(np.diff(ch[c].astype(np.int64), axis=0), axis=1)
        assert np.array_equal(plane, np.clip(d, 0, 255))
    # Gabor channels use the full [0,255] range after min-max normalisation
    for c in range(1, 36):
        plane = np.diff(np.diff(ch[c].astype(np.int64), axis=0), axis=1)
        assert plane.min() == 0 and plane.max() == 255


@pytest.mark.parametrize("index", [0, 6, 7, 20, 34])
def test_gabor_bank(oracle_mod, index):
    re, im = oracle_mod.gabor_kernel(index)
    assert re.shape[0] == [7, 9, 13, 19, 25][index // 7]
    assert np.array_equal(re, re[::-1, ::-1]) and np.array_equal(im, -im[::-1, ::-1])


@pytest.mark.parametrize("index", [3] + list(range(7, 35)))
def test_gabor_magnitude_vs_float64_correlation(oracle_mod, index):
    """The restated float32 correlation equals a float64 reference correlation (filter2D
    semantics: correlation, centred anchor, BORDER_REFLECT_101) to float32 rounding."""
    rng = np.random.default_rng(index)
    face = rng.integers(0, 256, (70, 64), dtype=np.uint8)
    re, im = oracle_mod.gabor_kernel(index)
    R = re.shape[0] // 2
    p = np.pad(face.astype(np.float64), R, mode="reflect")
    r = correlate2d(p, re.astype(np.float64), mode="valid")
    i = correlate2d(p, im.astype(np.float64), mode="valid")
    ref = np.sqrt(r * r + i * i)
    got = oracle_mod.gabor_mag(face, index)
    assert np.allclose(got, ref, rtol=2e-5, atol=2e-3 * ref.max() * 1e-2)


def test_threaded_equals_serial(oracle_mod):
    c = crops(2, seed=9)
    for img in c:
        a, ta = oracle_mod.analyze_face(img, (0, 0, 150, 150), threads=1, trace=True)
        b, tb = oracle_mod.analyze_face(img, (0, 0, 150, 150), threads=8, trace=True)
        assert np.array_equal(a["points"], b["points"]) and a["headpose"] == b["headpose"]
        assert np.array_equal(ta["mp_leaves"], tb["mp_leaves"])


def test_accuracy_band_on_bundled_faces(oracle_mod, fixtures):
    """eval_ffd's metric (eval_ffd.cpp:33-46,102-108) on the 20 annotated faces the reference ships.
    Pinned to the restatement's measured result (mean 0.0747, 78.5 % < 0.1 IOD; the reference's
    published LFW-test figures are 0.078 / 79.4 %, output/errors.txt).  Per-face parity with the
    reference's own output is pinned in tests/test_reference_pins.py."""
    errs = []
    for img, box, parts in zip(fixtures["images"], fixtures["boxes"], fixtures["parts"]):
        f, _ = oracle_mod.analyze_face(img, tuple(int(v) for v in box), threads=8)
        iod = np.linalg.norm((parts[0] + parts[1]) / 2.0 - (parts[6] + parts[7]) / 2.0)
        errs.append(np.linalg.norm(parts - f["points"], axis=1) / iod)
    errs = np.array(errs)
    assert abs(errs.mean() - 0.07472) < 5e-5, errs.mean()
    assert (errs < 0.1).sum() == 157, (errs < 0.1).sum()  # 157 of 200 landmarks = 78.5 %


def test_rejects_box_outside_image(oracle_mod, fixtures):
    with pytest.raises(RuntimeError):
        oracle_mod.analyze_face(fixtures["images"][0], (200, 200, 100, 100))
