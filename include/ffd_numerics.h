/*
 * ffd_numerics.h — the numeric definitions shared by the CPU oracle and the
 * HIP kernels so both produce identical bits.
 *
 * The reference calls libm `exp` inside areaUnderCurve
 * (/root/reference/src/face_utils.cpp:304-323) and `expf` inside
 * MeanShift::getWeightedMean (/root/reference/include/MeanShift.hpp:106-135).
 * glibc's and the GPU's (ocml) exponentials are both faithful (<1 ulp) but not
 * bitwise identical, and the head-pose tree selection takes floor(area*20)
 * (FaceForest.cpp:243), so a 1-ulp difference could flip a tree choice.  The
 * restatement therefore DEFINES exp as the deterministic routines below
 * (Cody-Waite reduction + Taylor polynomial in explicit fma Horner steps),
 * used by both sides.  Their accuracy against libm is checked in
 * tests/test_numerics.py (exp: |err| <= 2 ulp; expf: <= 1 ulp of the float).
 *
 * Everything here is IEEE binary64/binary32 arithmetic with round-to-nearest
 * and no contraction; both the oracle (g++ -ffp-contract=off) and the kernels
 * (hipcc -ffp-contract=off) are compiled that way.
 */
#ifndef FFD_NUMERICS_H
#define FFD_NUMERICS_H

#if defined(__HIPCC__)
#define FFD_HD __host__ __device__ __forceinline__
#else
#define FFD_HD static inline
#endif

#ifdef __cplusplus
#include <cmath>
#define FFD_RINT(x) std::rint(x)
#define FFD_LDEXP(x, k) std::ldexp((x), (k))
#else
#include <math.h>
#define FFD_RINT(x) rint(x)
#define FFD_LDEXP(x, k) ldexp((x), (k))
#endif

#ifdef __cplusplus
#define FFD_FMA(a, b, c) std::fma((a), (b), (c))
#else
#define FFD_FMA(a, b, c) fma((a), (b), (c))
#endif

/* Cody-Waite reduction x = k ln2 + r, |r| <= ln2/2 (shared by both routines). */
FFD_HD double ffd_exp_reduce(double x, int* k) {
  const double log2e = 1.4426950408889634074;
  const double ln2_hi = 6.93147180369123816490e-01;   /* 0x3FE62E42FEE00000 */
  const double ln2_lo = 1.90821492927058770002e-10;   /* 0x3DEA39EF35793C76 */
  double kd = FFD_RINT(x * log2e);
  *k = (int)kd;
  double hi = x - kd * ln2_hi; /* exact: kd*ln2_hi has <= 43 significant bits */
  return hi - kd * ln2_lo;
}

/* exp(x) in binary64: degree-13 Taylor polynomial of the reduced argument, fma Horner steps. */
FFD_HD double ffd_exp(double x) {
  if (x != x) return x;                               /* NaN */
  if (x > 709.782712893384) return HUGE_VAL;           /* overflow */
  if (x < -745.1332191019412) return 0.0;              /* underflow */
  int k;
  const double r = ffd_exp_reduce(x, &k);
  double p = 1.0 / 6227020800.0;                      /* 1/13! */
  p = FFD_FMA(p, r, 1.0 / 479001600.0);               /* 1/12! */
  p = FFD_FMA(p, r, 1.0 / 39916800.0);                /* 1/11! */
  p = FFD_FMA(p, r, 1.0 / 3628800.0);                 /* 1/10! */
  p = FFD_FMA(p, r, 1.0 / 362880.0);                  /* 1/9!  */
  p = FFD_FMA(p, r, 1.0 / 40320.0);                   /* 1/8!  */
  p = FFD_FMA(p, r, 1.0 / 5040.0);                    /* 1/7!  */
  p = FFD_FMA(p, r, 1.0 / 720.0);                     /* 1/6!  */
  p = FFD_FMA(p, r, 1.0 / 120.0);                     /* 1/5!  */
  p = FFD_FMA(p, r, 1.0 / 24.0);                      /* 1/4!  */
  p = FFD_FMA(p, r, 1.0 / 6.0);                       /* 1/3!  */
  p = FFD_FMA(p, r, 0.5);                             /* 1/2!  */
  p = FFD_FMA(p, r, 1.0);
  p = FFD_FMA(p, r, 1.0);
  return FFD_LDEXP(p, k);
}

/* expf(x) in binary32 (MeanShift weights, MeanShift.hpp:106-135): the binary32 rounding of a
 * degree-11 Taylor evaluation in binary64 (truncation error < 1e-14 relative, so the result is
 * the correctly rounded expf except within 1e-14 of a rounding boundary). */
FFD_HD float ffd_expf(float xf) {
  const double x = (double)xf;
  if (x != x) return xf;                               /* NaN */
  if (x > 88.8) return HUGE_VALF;                      /* overflow */
  if (x < -104.0) return 0.0f;                         /* underflow (below the smallest subnormal) */
  int k;
  const double r = ffd_exp_reduce(x, &k);
  double p = 1.0 / 39916800.0;                         /* 1/11! */
  p = FFD_FMA(p, r, 1.0 / 3628800.0);
  p = FFD_FMA(p, r, 1.0 / 362880.0);
  p = FFD_FMA(p, r, 1.0 / 40320.0);
  p = FFD_FMA(p, r, 1.0 / 5040.0);
  p = FFD_FMA(p, r, 1.0 / 720.0);
  p = FFD_FMA(p, r, 1.0 / 120.0);
  p = FFD_FMA(p, r, 1.0 / 24.0);
  p = FFD_FMA(p, r, 1.0 / 6.0);
  p = FFD_FMA(p, r, 0.5);
  p = FFD_FMA(p, r, 1.0);
  p = FFD_FMA(p, r, 1.0);
  return (float)FFD_LDEXP(p, k);
}

/* ffd_expf for arguments x <= 0 (MeanShift's -d/lamda, d >= 0 finite): the same operations without
 * the NaN / overflow branches, which no such argument reaches, and with the underflow test as a
 * select (no divergent branch on the GPU).  Equal to ffd_expf(x) for every x <= 0, -0 and -inf
 * included (tests/test_numerics.py). */
FFD_HD float ffd_expf_nonpos(float xf) {
  const int under = xf < -104.0f;
  const double x = (double)(under ? -104.0f : xf);
  int k;
  const double r = ffd_exp_reduce(x, &k);
  double p = 1.0 / 39916800.0;                         /* 1/11! */
  p = FFD_FMA(p, r, 1.0 / 3628800.0);
  p = FFD_FMA(p, r, 1.0 / 362880.0);
  p = FFD_FMA(p, r, 1.0 / 40320.0);
  p = FFD_FMA(p, r, 1.0 / 5040.0);
  p = FFD_FMA(p, r, 1.0 / 720.0);
  p = FFD_FMA(p, r, 1.0 / 120.0);
  p = FFD_FMA(p, r, 1.0 / 24.0);
  p = FFD_FMA(p, r, 1.0 / 6.0);
  p = FFD_FMA(p, r, 0.5);
  p = FFD_FMA(p, r, 1.0);
  p = FFD_FMA(p, r, 1.0);
  const float e = (float)FFD_LDEXP(p, k);
  return under ? 0.0f : e;
}

/* log(x) in binary64 for finite x > 0 (the entropy terms of forest training, MPSample::entropie_parts,
 * /root/reference/src/MPSample.cpp:276-297): x = 2^k m with m in [sqrt(2)/2, sqrt(2)), f = m - 1,
 * s = f / (2 + f), log(m) = f - s (f - R(s^2)) with fdlibm's e_log.c minimax coefficients, only +, -,
 * *, / (no fma), so the oracle and the kernels produce the same bits; within 1 ulp of libm's log
 * (tests/test_numerics.py).  Subnormal x is scaled by 2^54 first. */
FFD_HD double ffd_log(double x) {
  const double ln2_hi = 6.93147180369123816490e-01;  /* 0x3FE62E42FEE00000 */
  const double ln2_lo = 1.90821492927058770002e-10;  /* 0x3DEA39EF35793C76 */
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
               Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  int k = 0;
  if (x < 2.2250738585072014e-308) { x = x * 18014398509481984.0; k = -54; } /* 2^54 */
  int e;
#ifdef __cplusplus
  double m = std::frexp(x, &e);  /* x = m 2^e, m in [0.5, 1): exact */
#else
  double m = frexp(x, &e);
#endif
  if (m < 0.70710678118654752440) { m = m + m; e -= 1; }
  k += e;
  const double f = m - 1.0;  /* exact (Sterbenz) */
  const double s = f / (2.0 + f), z = s * s, w = z * z;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  const double R = t2 + t1, hfsq = 0.5 * f * f, dk = (double)k;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

/* a / b for a divisor b whose reciprocal y = RN(1/b) is given: q = RN(a y), r = a - b q (exact with
 * an fma), RN(q + r y) (Markstein's correction).  It is the correctly rounded quotient whenever the
 * premises of Markstein's theorem hold (not for subnormal quotients: |a| <= 2^-100 divides
 * directly); tests/test_numerics.py checks it against IEEE division for
 * every finite binary32 a at b = 10 (MeanShiftOption::kernel_size's default, MeanShift.hpp:20), the
 * only divisor the kernels use it for. */
FFD_HD float ffd_div_rcp(float a, float b, float y) {
  if (!(a > 0x1p-100f || a < -0x1p-100f)) return a / b;  /* tiny |a| (subnormal quotients): IEEE division */
#ifdef __cplusplus
  const float q = a * y;
  const float r = std::fma(-q, b, a);
  return std::fma(r, y, q);
#else
  const float q = a * y;
  const float r = fmaf(-q, b, a);
  return fmaf(r, y, q);
#endif
}

/* ffd_div_rcp without its tiny-|a| branch (MeanShift's weights, k_meanshift / k_meanshift4): the same quotient for
 * |a| > 2^-100; for smaller |a| a quotient of magnitude at most 2^-100 or zero, whose ffd_expf_nonpos is exactly
 * 1.0f, as the IEEE quotient's is (tests/numerics/check_numerics.c "quot", every such a) — so the weight
 * w * expf(-d / lamda) is the same bits, with no divergent branch on the GPU. */
FFD_HD float ffd_div_rcp_fast(float a, float b, float y) {
#ifdef __cplusplus
  const float q = a * y;
  return std::fma(std::fma(-q, b, a), y, q);
#else
  const float q = a * y;
  return fmaf(fmaf(-q, b, a), y, q);
#endif
}

#endif /* FFD_NUMERICS_H */
