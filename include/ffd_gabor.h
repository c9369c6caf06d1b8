/*
 * ffd_gabor.h — the separable Gabor factors shared by the CPU oracle and the HIP engine
 * (host code only).
 *
 * The reference builds 35 complex Gabor kernels (FeatureChannelFactory.hpp:186-251):
 *   K(x, y) = (k^2/sigma^2) exp(-(x^2 + y^2) k^2 / (2 sigma^2)) * (exp(i k (x cos(phi) + y sin(phi))) - c),
 *   c = exp(-sigma^2 / 2), sigma = pi/2, k = (pi/2) / sqrt(2)^nu, phi = pi mu / 8,
 * and correlates the face with each (cv::filter2D).  For widths >= 9 (nu >= 1) OpenCV 2.4.9
 * evaluates that correlation through a DFT whose rounding cannot be reproduced without OpenCV,
 * so the restatement DEFINES those correlations by the exact factorisation
 *   (k^2/sigma^2) exp(-(x^2+y^2) k^2/(2 sigma^2)) = g(x) g(y),  g(t) = (k/sigma) exp(-t^2 k^2/(2 sigma^2))
 *   cos(a x + b y) = cos(a x) cos(b y) - sin(a x) sin(b y),  sin(a x + b y) = sin(a x) cos(b y) + cos(a x) sin(b y)
 * with a = k cos(phi), b = k sin(phi): a vertical 1-D pass (V planes) followed by a horizontal
 * 1-D pass per orientation.  Equal to the 2-D correlation in exact arithmetic (checked against a
 * float64 2-D correlation in tests/test_oracle.py); the fp32 operation order is fixed in
 * oracle/ffd_oracle.cpp gabor_sep_mag and reproduced by ffd_kernels.hip k_gabor_sep.
 *
 * cos(pi mu / 8) and sin(pi mu / 8) are taken from s_j = sin(j pi / 8), j = 0..4 (s_0 = 0,
 * s_4 = 1 exactly), so orientations that share |a| or b share the same factors:
 *   mu : 0      1       2       3       4      5        6
 *   |a|: k      k s3    k s2    k s1    0      k s1     k s2     -> horizontal set p = 0,1,2,3,4,3,2
 *   b  : 0      k s1    k s2    k s3    k      k s3     k s2     -> vertical set   q = 0,1,2,3,4,3,2
 *   sign(a): +  +       +       +       +      -        -
 * q = 0 is the plain Gaussian plane (b = 0); p = 4 is the plain Gaussian (a = 0).
 */
#ifndef FFD_GABOR_H
#define FFD_GABOR_H

#include <cmath>

#define FFD_GABOR_MAX_R 12

typedef struct {
  int R;                                     /* half width: kernel width 2R+1 */
  float c;                                   /* exp(-sigma^2/2) as float */
  float g[FFD_GABOR_MAX_R + 1];              /* g(t), t = 0..R */
  float vc[4][FFD_GABOR_MAX_R + 1];          /* q = 1..4: g(t) cos(b_q t) */
  float vs[4][FFD_GABOR_MAX_R + 1];          /* q = 1..4: g(t) sin(b_q t) (vs[.][0] = 0) */
  float hc[5][FFD_GABOR_MAX_R + 1];          /* p = 0..4: g(t) cos(a_p t) (hc[4] = g) */
  float hs[5][FFD_GABOR_MAX_R + 1];          /* p = 0..4: g(t) sin(a_p t), t >= 0 (odd in t) */
} ffd_gabor_sep;

/* orientation mu -> horizontal set p, vertical set q, sign of a */
static const int FFD_GABOR_P[7] = {0, 1, 2, 3, 4, 3, 2};
static const int FFD_GABOR_Q[7] = {0, 1, 2, 3, 4, 3, 2};
static const int FFD_GABOR_SGN[7] = {1, 1, 1, 1, 1, -1, -1};

/* Factors of scale nu = 1..4, in the reference's parameterisation (createKernel,
 * FeatureChannelFactory.hpp:186-205; initGaborKernels :234-251). */
static inline void ffd_gabor_sep_init(int nu, ffd_gabor_sep* s) {
  const double CV_PI = 3.1415926535897932384626433832795;
  const double sigma = 1.0 / 2.0 * CV_PI, F = std::sqrt(2.0);
  const double k = (CV_PI / 2) / std::pow(F, (double)nu);
  double width = std::round((sigma / k) * 6 + 1);
  if (std::fmod(width, 2.0) == 0.0) width++;
  const int R = (int)((width - 1) / 2);
  s->R = R;
  s->c = (float)std::exp(-(std::pow(sigma, 2) / 2));
  double sj[5];
  sj[0] = 0.0;
  for (int j = 1; j < 4; j++) sj[j] = std::sin(CV_PI * j / 8);
  sj[4] = 1.0;
  const double a[5] = {k * sj[4], k * sj[3], k * sj[2], k * sj[1], 0.0};
  const double b[4] = {k * sj[1], k * sj[2], k * sj[3], k * sj[4]};
  for (int t = 0; t <= FFD_GABOR_MAX_R; t++) {
    const bool in = t <= R;
    const double gd = (k / sigma) * std::exp(-std::pow((double)t, 2) * std::pow(k, 2) / (2 * std::pow(sigma, 2)));
    s->g[t] = in ? (float)gd : 0.f;
    for (int q = 0; q < 4; q++) {
      s->vc[q][t] = in ? (float)(gd * std::cos(b[q] * t)) : 0.f;
      s->vs[q][t] = in ? (float)(gd * std::sin(b[q] * t)) : 0.f;
    }
    for (int p = 0; p < 5; p++) {
      s->hc[p][t] = in ? (float)(gd * std::cos(a[p] * t)) : 0.f;
      s->hs[p][t] = in ? (float)(gd * std::sin(a[p] * t)) : 0.f;
    }
  }
}

/* The reference's 2-D kernel of scale nu, orientation mu (createKernel, FeatureChannelFactory.hpp:186-205)
 * as floats, [row j = y + R][column i = x + R]; returns the width 2R + 1 (re / im hold width^2 taps). */
static inline int ffd_gabor_taps(int nu, int mu, float* re, float* im) {
  const double CV_PI = 3.1415926535897932384626433832795;
  const double sigma = 1.0 / 2.0 * CV_PI, F = std::sqrt(2.0);
  const double k = (CV_PI / 2) / std::pow(F, (double)nu), phi = CV_PI * mu / 8;
  double width = std::round((sigma / k) * 6 + 1);
  if (std::fmod(width, 2.0) == 0.0) width++;
  const int W = (int)width, off = (int)((width - 1) / 2);
  for (int i = 0; i < W; i++)
    for (int j = 0; j < W; j++) {
      const int x = i - off, y = j - off;
      const double t1 = (std::pow(k, 2) / std::pow(sigma, 2)) *
                        std::exp(-(std::pow((double)x, 2) + std::pow((double)y, 2)) * std::pow(k, 2) / (2 * std::pow(sigma, 2)));
      const double t2 = std::cos(k * std::cos(phi) * x + k * std::sin(phi) * y) - std::exp(-(std::pow(sigma, 2) / 2));
      const double t3 = std::sin(k * std::cos(phi) * x + k * std::sin(phi) * y);
      re[j * W + i] = (float)(t1 * t2);
      im[j * W + i] = (float)(t1 * t3);
    }
  return W;
}

#endif /* FFD_GABOR_H */
