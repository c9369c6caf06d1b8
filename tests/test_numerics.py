"""Numeric premises the restatement and the kernels rely on (CPU-only)."""
import math

import numpy as np
import pytest


def test_float_division_truncation_equals_integer_division():
    """ImageSample::evalTest computes p = (int)(R / (float)(w*h)) (ImageSample.cpp:347,353); the
    kernels use the exact integer quotient.  Equal for every rectangle sum R in [0, 255*484] and
    area in [1, 484] (rect sides 1..22)."""
    R = np.arange(0, 255 * 484 + 1, dtype=np.int64)
    Rf = R.astype(np.float32)
    for a in range(1, 485):
        q = (Rf / np.float32(a)).astype(np.int64)  # IEEE float32 division, then trunc toward 0
        assert np.array_equal(q, R // a), a


def test_rcp_fma_division_equals_integer_division():
    """The traversal kernel (ffd_kernels.hip rect_mean_walk) computes the quotient as
    (int)fma((float)R, rcp(area), 0.00075) with the hardware reciprocal; equal to R // area for
    every R in [0, 255*area], area in [1, 484], for any reciprocal within 2 ulp of 1/area.
    fma is emulated exactly: R * r + eps needs <= 48 significant bits, so float64 holds it exactly
    and one rounding to float32 is the fused result."""
    eps = np.float64(np.float32(0.00075))
    for a in range(1, 485):
        R = np.arange(0, 255 * a + 1, dtype=np.float64)
        r0 = np.float32(1.0) / np.float32(a)
        rs = [r0]
        for d in (np.float32(np.inf), np.float32(0.0)):
            r = r0
            for _ in range(2):
                r = np.nextafter(r, d)
                rs.append(r)
        for r in rs:
            q = (R * np.float64(r) + eps).astype(np.float32).astype(np.int64)
            assert np.array_equal(q, np.arange(0, 255 * a + 1) // a), (a, r)


def test_ffd_exp_matches_libm(oracle_mod):
    """ffd_exp (include/ffd_numerics.h) is within 2 ulp of libm exp over the argument ranges the
    path uses (areaUnderCurve: -0.5 t^2 <= 0; MeanShift: -d/10 in [-30, 0])."""
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.uniform(-745, 709, 4000), rng.uniform(-40, 0, 4000), rng.uniform(-1, 1, 2000),
                         [0.0, -0.0, 1e-300, -1e-300, 709.7, -708.3, -744.0]])
    for x in xs:
        got, ref = oracle_mod.exp(float(x)), math.exp(float(x))
        if ref == 0.0 or got == 0.0:
            assert abs(got - ref) <= 5e-324 * 4
            continue
        ulp = math.ulp(ref)
        if ref < 2.2250738585072014e-308:  # subnormal results: absolute tolerance
            assert abs(got - ref) <= 2 * 5e-324
        else:
            assert abs(got - ref) <= 2 * ulp, (x, got, ref)
    assert math.isnan(oracle_mod.exp(float("nan")))
    assert oracle_mod.exp(-1e6) == 0.0 and oracle_mod.exp(1e6) == math.inf


def test_ffd_expf_within_one_ulp_of_correctly_rounded(oracle_mod):
    """ffd_expf (MeanShift weights) is within 1 ulp of the correctly rounded binary32 exp over the
    MeanShift argument range -d/10, d in [0, 400], and a few wider points."""
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(-40, 0, 20000), rng.uniform(-103, 88, 2000), [0.0, -1e-7, -87.0]])
    for x in xs.astype(np.float32):
        got = np.float32(oracle_mod.expf(float(x)))
        ref = np.float32(math.exp(float(x)))  # float64 exp, then one rounding to float32
        if ref == 0 or got == 0:
            assert abs(float(got) - float(ref)) <= 2 * 1.4e-45
            continue
        assert abs(float(got) - float(ref)) <= float(np.spacing(ref)), (x, got, ref)


def test_sqrt_2pi_literal():
    assert 2.5066282746310002 == math.sqrt(2 * math.pi)


def test_area_under_curve_partition(oracle_mod):
    """areaUnderCurve (face_utils.cpp:304-323) over the 5 pose bins of FaceForest.cpp:216-222
    integrates the Gaussian: for a moderate sigma the bins sum to ~1 (left Riemann sums)."""
    poseT = np.array([-2.5, -0.35, -0.20, 0.20, 0.35, 2.5], np.float32)
    for mean, std in [(0.0, 0.4), (0.3, 0.2), (-1.0, 0.5)]:
        s = sum(oracle_mod.area_under_curve(float(poseT[j]), float(poseT[j + 1]), mean, std) for j in range(5))
        assert abs(s - 1.0) < 0.03, (mean, std, s)


@pytest.mark.parametrize("w", [7, 9, 13, 19, 25])
def test_gabor_flop_model(w):
    import bench
    assert bench.gabor_flops_per_pixel(w) > 0


def _run_numerics_check(which):
    """Build and run tests/numerics/check_numerics.c (exhaustive, multi-threaded C; see its header)."""
    import os
    import subprocess
    import tempfile
    here = os.path.dirname(os.path.abspath(__file__))
    src = os.path.join(here, "numerics", "check_numerics.c")
    exe = os.path.join(tempfile.mkdtemp(prefix="ffd_num_"), "check_numerics")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, src, "-lm", "-lpthread"], check=True)
    out = subprocess.run([exe, which], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout


def test_markstein_division_by_ten_is_ieee_division():
    """ffd_div_rcp(a, 10, RN(1/10)) == a / 10 for every finite binary32 a (the MeanShift weight's
    -d/lamda at the default kernel_size, MeanShift.hpp:20,123; k_meanshift's fast quotient)."""
    _run_numerics_check("div")


def test_fast_quotient_gives_the_same_weight():
    """ffd_div_rcp_fast (no tiny-|a| branch; k_meanshift's quotient) gives the same ffd_expf_nonpos as IEEE -d / 10 for
    every binary32 d in [0, 2^-100]; above it the quotients are equal (the "div" check)."""
    _run_numerics_check("quot")


def test_expf_nonpos_equals_expf():
    """ffd_expf_nonpos == ffd_expf bitwise for every binary32 x in [-110, 0] (and -inf, -1e30)."""
    _run_numerics_check("exp")
