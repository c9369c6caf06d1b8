"""Float-integral rectangle halves past 2^27.

A face or image sample whose CV_32F integrals reach 2^24 (FaceDesc::fint; OpenCV's integral_ rounds there,
FeatureChannelFactory.hpp:46-57) keeps them modulo 2^16, and rect_mean_fint (ffd_kernels.hip) recovers every
rectangle half's four-corner combination in a window of 2^16 values.  Round 5's window [-128, 65407] was sized for
integrals below 2^27.  Faces now go up to FINT_LIMIT = 2^31, where a half's rounding error reaches 2 x 11 x 64 = 1,408,
so the window is [-2048, 63488).  Faces and samples at or past 2^31 are refused (FFD_ERR_UNSUPPORTED).

CPU: a numpy restatement of integral_'s float accumulation (`s += src[x]; sum[x] = sum[x - step] + s`, every add
rounded to binary32), pinned to the oracle's channel 0 on a small tall face, on a 125 x 17,400 face: bright rows
above, dark sparse noise below, so rectangle halves with true sums near 0 sit at integrals near 2^29.  The old window
mis-recovers hundreds of them; the new one recovers every one.  GPU: the same face as an ImageSample; its head-pose
and FFD leaves at patches inside the dark region equal the oracle's, and a sample past 2^31 is refused."""
import numpy as np
import pytest

import face_alignment_cvpr_2012_amd as ffd

W, TOP, BOT, LB = 125, 17000, 400, 40


def tall_face(top=TOP, bot=BOT, lb=LB, seed=3):
    """Bright rows [0, top); below, columns [0, lb) bright and the rest sparse noise in {0, 1, 2, 3}."""
    rng = np.random.default_rng(seed)
    g = np.zeros((top + bot, W), np.uint8)
    g[:top] = 255
    g[top:, :lb] = 255
    g[top:, lb:] = (rng.random((bot, W - lb)) < 0.05) * rng.integers(1, 4, (bot, W - lb))
    return g


def float_integral(g):
    """integral_ with a float sum (OpenCV 2.4.9 imgproc/sumpixels.cpp as the oracle restates it)."""
    h, w = g.shape
    out = np.zeros((h + 1, w + 1), np.float32)
    for y in range(h):
        s = np.cumsum(g[y].astype(np.float32), dtype=np.float32)  # row prefix: exact (< 2^24)
        out[y + 1, 1:] = out[y, 1:] + s  # one binary32 rounding per add
    return out


def recover(v, lo):
    """rect_mean_fint's half: the four-corner combination modulo 2^16, read in the window [lo, lo + 65536)."""
    m = v & 0xFFFF
    return np.where(m >= 65536 + lo, m - 65536, m)


def test_float_integral_restatement_matches_oracle(oracle_mod):
    g = tall_face(top=1500, bot=500)
    ch = oracle_mod.channels(g)
    got = float_integral(g)
    assert got.max() >= 2 ** 24  # past 2^24: the float integral rounds
    assert np.array_equal(ch[0].astype(np.int64), got.astype(np.int64))


def test_window_recovers_every_half_past_2_27():
    g = tall_face()
    I = float_integral(g).astype(np.int64)
    assert 2 ** 29 <= I.max() < 2 ** 31
    rng = np.random.default_rng(11)
    n = 300_000
    ws, hs = rng.integers(1, 23, n), rng.integers(1, 12, n)  # a half: <= 22 columns, <= 11 rows
    xs = rng.integers(LB, W - ws + 1)
    ys = rng.integers(TOP + 1, g.shape[0] - 12, n)
    v = I[ys + hs, xs + ws] - I[ys, xs + ws] - I[ys + hs, xs] + I[ys, xs]
    assert v.min() < -128  # the rounding pushes near-zero halves below round 5's window
    assert np.abs(v - np.clip(v, 0, 61710)).max() <= 1408  # inside the stated error bound
    assert (recover(v, -128) != v).sum() > 100  # round 5's window mis-recovers them
    assert np.array_equal(recover(v, -2048), v)  # the window in use recovers every one


@pytest.mark.gpu
def test_tall_sample_dark_rectangles_match_oracle(engine, oracle_mod):
    g = tall_face()
    ch = oracle_mod.channels(g)
    rng = np.random.default_rng(5)
    n = 400
    xy = np.stack([rng.integers(0, W - 31 + 1, n), rng.integers(TOP - 8, g.shape[0] - 31 + 1, n)], 1).astype(np.int32)
    trees = list(range(0, 100, 5))
    want_hp = oracle_mod.eval_patches(ch, xy, ffd.FOREST_HEADPOSE, list(range(15)))
    want_mp = oracle_mod.eval_patches(ch, xy, ffd.FOREST_FFD, trees)
    with ffd.ImageSample(engine, g) as s:
        assert np.array_equal(s.eval_leaves(ffd.FOREST_HEADPOSE, xy, list(range(15))), want_hp)
        assert np.array_equal(s.eval_leaves(ffd.FOREST_FFD, xy, trees), want_mp)
    assert np.array_equal(ffd.Forest(engine, ffd.FOREST_FFD).evaluate(ch, xy, trees), want_mp)


@pytest.mark.gpu
def test_sample_past_2_31_is_refused(engine):
    h = (2 ** 31) // (255 * W) + 1  # 255 W h >= 2^31
    with pytest.raises(ffd.FFDError) as e:
        ffd.ImageSample(engine, np.zeros((h, W), np.uint8))
    assert e.value.status == ffd.STATUS_UNSUPPORTED
