// ffd_oracle.cpp — CPU restatement of the reference hot path. TEST INFRASTRUCTURE.
//
// This file is the parity oracle for the HIP engine: a plain C++17 (no OpenCV,
// no Boost) restatement of FaceForest::analyzeFace and everything below it, in
// reference order, with the numeric semantics of SURVEY.md Appendix B.  Only
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
//
// Parity status:
//   * PINNED  — model loader: node/leaf counts and threshold sums of every tree
//               equal the known-answer values computed from the reference's own
//               archives (tests/test_model.py).
//   * SANITY  — end-to-end accuracy on the 20 annotated faces the reference
//               ships (data/imgs/index_random_subset.txt) is checked against
//               the band of the reference's published errors (output/errors.txt).
//   * UNPINNED — every value at the OpenCV 2.4.9 boundary (cvtColor, resize,
//               filter2D, normalize, convertTo, Sobel, cvRound): OpenCV is not
//               in this image and the reference ships no intermediate values,
//               so these follow OpenCV 2.4.9's documented/x86-SSE2 behaviour as
//               restated here ("parity unpinned" for channel values and exact
//               landmark positions).
//
// Reference files followed (paths relative to /root/reference):
//   src/FaceForest.cpp:183-258           analyzeFace
//   src/face_utils.cpp:183-323           getHeadPoseVotesMT, getFacialFeaturesVotesMT, areaUnderCurve
//   include/MeanShift.hpp:16-135         MeanShift
//   src/ImageSample.cpp:11-90            ImageSample, evalTest (integral branch)
//   include/FeatureChannelFactory.hpp:35-286  channels, Gabor kernels
//   include/Forest.hpp:80-90, Tree.hpp:173-191, TreeNode.hpp:54-66,129-136  traversal
//   src/MPSample.cpp:77-84, src/HeadPoseSample.cpp:39-46  eval: test <= threshold -> left
//   include/FaceForest.hpp:34-58, include/Constants.hpp:24-30,65-68  options/constants
//   include/ThreadPool.hpp:24-64         per-call pools (CPU-baseline shape)
#include "ffd_oracle.h"
#include "ffd_gabor.h"

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../include/ffd_model_format.h"
#include "../include/ffd_numerics.h"

namespace {

thread_local std::string g_err;

// ------------------------------------------------------------------ model ----
struct Node {           // TreeNode<S> (TreeNode.hpp:138-146), pointer-free
  int32_t left = -1, right = -1, leaf = -1;
  int16_t ch = 0, r1[4] = {0, 0, 0, 0}, r2[4] = {0, 0, 0, 0};
  int32_t thr = 0;
};

struct Forest {
  std::vector<int32_t> roots;  // global node index of each tree's root
  std::vector<Node> nodes;
  int ntrees_per_forest = 0, n_forests = 0, face_size = 125;
  float patch_ratio = 0.25f;
  // HP leaf payload
  std::vector<int32_t> hp_n, hp_labels;
  std::vector<float> hp_fg;
  // MP leaf payload
  std::vector<int32_t> mp_n;
  std::vector<float> mp_fg, mp_var, mp_pf;
  std::vector<int16_t> mp_off;
};

Forest g_hp, g_mp;
bool g_loaded = false;
std::mutex g_mu;

struct Arr {
  std::string dtype;
  std::vector<uint64_t> shape;
  std::vector<uint8_t> data;
  template <class T> const T* p() const { return (const T*)data.data(); }
  uint64_t n() const { uint64_t v = 1; for (auto s : shape) v *= s; return v; }
};

std::map<std::string, Arr> read_container(const char* path) {
  FILE* f = std::fopen(path, "rb");
  if (!f) throw std::runtime_error(std::string("cannot open ") + path);
  char magic[8];
  uint32_t ver, n;
  if (std::fread(magic, 1, 8, f) != 8 || std::memcmp(magic, FFD_MODEL_MAGIC, 8) ||
      std::fread(&ver, 4, 1, f) != 1 || std::fread(&n, 4, 1, f) != 1 || ver != FFD_MODEL_VERSION) {
    std::fclose(f);
    throw std::runtime_error("bad model header");
  }
  std::vector<ffd_array_entry> e(n);
  if (std::fread(e.data(), sizeof(ffd_array_entry), n, f) != n) { std::fclose(f); throw std::runtime_error("bad model table"); }
  std::map<std::string, Arr> out;
  for (auto& x : e) {
    Arr a;
    a.dtype = x.dtype;
    for (uint32_t i = 0; i < x.ndim; i++) a.shape.push_back(x.shape[i]);
    a.data.resize(x.nbytes);
    std::fseek(f, (long)x.offset, SEEK_SET);
    if (x.nbytes && std::fread(a.data.data(), 1, x.nbytes, f) != x.nbytes) { std::fclose(f); throw std::runtime_error("truncated model"); }
    out[std::string(x.name)] = std::move(a);
  }
  std::fclose(f);
  return out;
}

// Rebuild pointer structure from pre-order records (TreeNode::serialize order:
// node, then full left subtree, then right subtree; TreeNode.hpp:150-164).
void build_forest(const std::map<std::string, Arr>& m, const std::string& p, Forest& F, bool hp) {
  auto get = [&](const std::string& k) -> const Arr& {
    auto it = m.find(p + "." + k);
    if (it == m.end()) throw std::runtime_error("missing array " + p + "." + k);
    return it->second;
  };
  const Arr& prm = get("param");
  F.ntrees_per_forest = prm.p<int32_t>()[3];
  F.face_size = prm.p<int32_t>()[6];
  F.n_forests = prm.p<int32_t>()[7];
  F.patch_ratio = get("patch_ratio").p<float>()[0];
  const Arr& off = get("tree_node_off");
  const Arr& nl = get("node_leaf");
  const Arr& ns = get("node_split");
  uint64_t T = off.n() - 1, N = nl.n();
  F.nodes.assign(N, Node());
  F.roots.clear();
  for (uint64_t t = 0; t < T; t++) {
    int64_t b = off.p<int64_t>()[t], e = off.p<int64_t>()[t + 1];
    F.roots.push_back((int32_t)b);
    std::vector<int64_t> stack;  // nodes awaiting children
    for (int64_t i = b; i < e; i++) {
      Node& nd = F.nodes[i];
      const int16_t* s = ns.p<int16_t>() + i * FFD_SPLIT_FIELDS;
      nd.leaf = nl.p<int32_t>()[i];
      nd.ch = s[0];
      for (int k = 0; k < 4; k++) { nd.r1[k] = s[1 + k]; nd.r2[k] = s[5 + k]; }
      nd.thr = s[9];
      if (i > b) {  // attach to the most recent parent still missing a child
        if (stack.empty()) throw std::runtime_error("malformed pre-order tree");
        Node& par = F.nodes[stack.back()];
        if (par.left < 0) par.left = (int32_t)i;
        else { par.right = (int32_t)i; stack.pop_back(); }
      }
      if (nd.leaf < 0) stack.push_back(i);
    }
    if (!stack.empty()) throw std::runtime_error("incomplete tree");
  }
  if (hp) {
    const Arr& n = get("leaf_n"); const Arr& fg = get("leaf_fg"); const Arr& lb = get("leaf_labels");
    F.hp_n.assign(n.p<int32_t>(), n.p<int32_t>() + n.n());
    F.hp_fg.assign(fg.p<float>(), fg.p<float>() + fg.n());
    F.hp_labels.assign(lb.p<int32_t>(), lb.p<int32_t>() + lb.n());
  } else {
    const Arr& n = get("leaf_n"); const Arr& fg = get("leaf_fg"); const Arr& o = get("leaf_offset");
    const Arr& v = get("leaf_var"); const Arr& pf = get("leaf_pf");
    F.mp_n.assign(n.p<int32_t>(), n.p<int32_t>() + n.n());
    F.mp_fg.assign(fg.p<float>(), fg.p<float>() + fg.n());
    F.mp_off.assign(o.p<int16_t>(), o.p<int16_t>() + o.n());
    F.mp_var.assign(v.p<float>(), v.p<float>() + v.n());
    F.mp_pf.assign(pf.p<float>(), pf.p<float>() + pf.n());
  }
}

// ------------------------------------------------------------ thread pool ----
// Per-call pool of n threads, one task per unit, joined before returning —
// the shape of boost::thread_pool::ThreadPool (ThreadPool.hpp:24-64) at its
// call sites FeatureChannelFactory.hpp:82-86 and face_utils.cpp:210-216,267-274.
void run_pool(int threads, int ntasks, const std::function<void(int)>& fn) {
  if (threads <= 1) {
    for (int i = 0; i < ntasks; i++) fn(i);
    return;
  }
  std::atomic<int> next{0};
  std::vector<std::thread> pool;
  pool.reserve(threads);
  for (int t = 0; t < threads; t++)
    pool.emplace_back([&] {
      for (;;) {
        int i = next.fetch_add(1);
        if (i >= ntasks) break;
        fn(i);
      }
    });
  for (auto& th : pool) th.join();
}

// ---------------------------------------------------------- OpenCV 2.4.9 ----
inline int cv_round(float v) {  // cvRound: SSE2 cvtss2si, round-half-even; NaN/overflow -> INT_MIN
  if (!(v >= -2147483648.0f && v < 2147483648.0f)) return INT_MIN;
  return (int)std::nearbyint(v);
}
inline int cv_round_d(double v) {
  if (!(v >= -2147483648.0 && v < 2147483648.0)) return INT_MIN;
  return (int)std::nearbyint(v);
}
inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }
inline int16_t sat_s16(int v) { return (int16_t)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }
inline int cv_floor(double v) { return (int)std::floor(v); }
inline int reflect101(int i, int n) {  // BORDER_REFLECT_101 for n >= 2
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}

// cvtColor(BGR2GRAY) 8U: fixed point, yuv_shift 14 (B 1868, G 9617, R 4899).
inline uint8_t gray_px(const uint8_t* p) {
  return (uint8_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + (1 << 13)) >> 14);
}

// resize(INTER_LINEAR) 8U, OpenCV 2.4.9 resizeGeneric_ with HResizeLinear<uchar,int,short,2048>
// and VResizeLinear<uchar,int,short,FixedPtCast<int,uchar,22>, VResizeLinearVec_32s8u> (SSE2).
// Exact 2x down-scales take the INTER_AREA fast path; equal sizes copy.
void cv_resize(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh) {
  if (sw == dw && sh == dh) {
    for (int y = 0; y < dh; y++) std::memcpy(dst + y * dw, src + y * sstride, dw);
    return;
  }
  double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
  double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
  int iscale_x = (int)cv_round_d(scale_x), iscale_y = (int)cv_round_d(scale_y);
  bool is_area_fast = std::fabs(scale_x - iscale_x) < DBL_EPSILON && std::fabs(scale_y - iscale_y) < DBL_EPSILON;
  if (is_area_fast && iscale_x == 2 && iscale_y == 2) {
    // resizeAreaFast_ 2x2: (a+b+c+d+2)>>2
    for (int y = 0; y < dh; y++)
      for (int x = 0; x < dw; x++) {
        const uint8_t* s0 = src + (2 * y) * sstride + 2 * x;
        const uint8_t* s1 = s0 + sstride;
        dst[y * dw + x] = (uint8_t)((s0[0] + s0[1] + s1[0] + s1[1] + 2) >> 2);
      }
    return;
  }
  const int ONE = 2048;
  std::vector<int> xofs(dw), yofs(dh);
  std::vector<int16_t> ialpha(dw * 2), ibeta(dh * 2);
  int xmax = dw;
  for (int dx = 0; dx < dw; dx++) {
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = cv_floor(fx);
    fx -= sx;
    if (sx < 0) fx = 0, sx = 0;
    if (sx + 1 >= sw) {
      xmax = std::min(xmax, dx);
      if (sx >= sw - 1) fx = 0, sx = sw - 1;
    }
    xofs[dx] = sx;
    ialpha[dx * 2] = sat_s16(cv_round((1.f - fx) * ONE));
    ialpha[dx * 2 + 1] = sat_s16(cv_round(fx * ONE));
  }
  for (int dy = 0; dy < dh; dy++) {  // rows are NOT clamped here; resizeGeneric_ clips row indices
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    int sy = cv_floor(fy);
    fy -= sy;
    yofs[dy] = sy;
    ibeta[dy * 2] = sat_s16(cv_round((1.f - fy) * ONE));
    ibeta[dy * 2 + 1] = sat_s16(cv_round(fy * ONE));
  }
  // columns covered by the SSE2 vertical pass (VResizeLinearVec_32s8u loop bounds)
  int xv = 0;
  while (xv <= dw - 16) xv += 16;
  while (xv < dw - 4) xv += 4;
  std::vector<int> r0(dw), r1(dw);
  auto hresize = [&](const uint8_t* S, int* D) {
    int dx = 0;
    for (; dx < xmax; dx++) D[dx] = S[xofs[dx]] * ialpha[dx * 2] + S[xofs[dx] + 1] * ialpha[dx * 2 + 1];
    for (; dx < dw; dx++) D[dx] = S[xofs[dx]] * ONE;
  };
  for (int dy = 0; dy < dh; dy++) {
    // clip(sy0 - ksize2 + 1 + k, 0, sh) for k = 0, 1
    int sy0 = std::max(0, std::min(yofs[dy], sh - 1));
    int sy1 = std::max(0, std::min(yofs[dy] + 1, sh - 1));
    hresize(src + sy0 * sstride, r0.data());
    hresize(src + sy1 * sstride, r1.data());
    int b0 = ibeta[dy * 2], b1 = ibeta[dy * 2 + 1];
    uint8_t* D = dst + dy * dw;
    for (int x = 0; x < dw; x++) {
      if (x < xv) {
        // _mm_packs_epi32(srai(S,4)) -> _mm_mulhi_epi16 -> _mm_adds_epi16 -> +2 >> 2 -> packus
        int s0 = std::max(-32768, std::min(32767, r0[x] >> 4));
        int s1 = std::max(-32768, std::min(32767, r1[x] >> 4));
        int m0 = (s0 * b0) >> 16, m1 = (s1 * b1) >> 16;
        int a = std::max(-32768, std::min(32767, m0 + m1));
        a = std::max(-32768, std::min(32767, a + 2)) >> 2;
        D[x] = sat_u8(a);
      } else {
        D[x] = sat_u8((b0 * r0[x] + b1 * r1[x] + (1 << 21)) >> 22);
      }
    }
  }
}

// cv::integral(img, sum, CV_32F): OpenCV 2.4.9 integral_<uchar, float, double> accumulates in float,
// s += src[x]; sum[x] = sum[x - sumstep] + s (every add rounded), so once a value passes 2^24 (a tall
// face: 255 W H >= 2^24) the integral is rounded; below that it is the exact integer sum.  Stored as
// u32 (every value is an integer-valued float < 2^32).
void integral(const uint8_t* img, int w, int h, uint32_t* out) {
  int W1 = w + 1;
  for (int x = 0; x <= w; x++) out[x] = 0;
  for (int y = 0; y < h; y++) {
    float s = 0;
    out[(y + 1) * W1] = 0;
    for (int x = 0; x < w; x++) {
      s += img[y * w + x];
      out[(y + 1) * W1 + x + 1] = (uint32_t)((float)out[y * W1 + x + 1] + s);
    }
  }
}

// ------------------------------------------------------------ Gabor bank ----
struct GaborKernel { int width; std::vector<float> re, im; };  // [row j = y+off][col i = x+off]
std::vector<GaborKernel> g_gabor;

// FeatureChannelFactory::createKernel / initGaborKernels (FeatureChannelFactory.hpp:186-251)
void init_gabor() {
  if (!g_gabor.empty()) return;
  const double CV_PI = 3.1415926535897932384626433832795;
  double sigma = 1.0 / 2.0 * CV_PI;
  double dF = std::sqrt(2.0);
  for (int iNu = 0; iNu <= 4; iNu++)
    for (int iMu = 0; iMu < 7; iMu++) {
      double F = dF;
      double k = (CV_PI / 2) / std::pow(F, (double)iNu);
      double phi = CV_PI * iMu / 8;
      double width = std::round((sigma / k) * 6 + 1);
      if (std::fmod(width, 2.0) == 0.0) width++;
      GaborKernel g;
      g.width = (int)width;
      g.re.assign(g.width * g.width, 0.f);
      g.im.assign(g.width * g.width, 0.f);
      int off_set = (int)((width - 1) / 2);
      for (int i = 0; i < g.width; i++)
        for (int j = 0; j < g.width; j++) {
          int x = i - off_set, y = j - off_set;
          double dTemp1 = (std::pow(k, 2) / std::pow(sigma, 2)) *
                          std::exp(-(std::pow((double)x, 2) + std::pow((double)y, 2)) * std::pow(k, 2) /
                                   (2 * std::pow(sigma, 2)));
          double dTemp2 = std::cos(k * std::cos(phi) * x + k * std::sin(phi) * y) - std::exp(-(std::pow(sigma, 2) / 2));
          double dTemp3 = std::sin(k * std::cos(phi) * x + k * std::sin(phi) * y);
          g.re[j * g.width + i] = (float)(dTemp1 * dTemp2);
          g.im[j * g.width + i] = (float)(dTemp1 * dTemp3);
        }
      // point symmetry required by the folded correlation below
      int n = g.width * g.width;
      for (int t = 0; t < n; t++)
        if (g.re[t] != g.re[n - 1 - t] || g.im[t] != -g.im[n - 1 - t])
          throw std::runtime_error("Gabor kernel not point-symmetric");
      g_gabor.push_back(std::move(g));
    }
}

// Separable factors of scales nu = 1..4 (include/ffd_gabor.h).
const ffd_gabor_sep& gabor_sep(int nu) {
  static ffd_gabor_sep tab[5];
  static std::once_flag once;
  std::call_once(once, [] {
    for (int v = 1; v <= 4; v++) ffd_gabor_sep_init(v, &tab[v]);
  });
  return tab[nu];
}

// >= 9x9 kernels (DEFINED, see include/ffd_gabor.h): the exact separable factorisation.
//  V pass (down each column, reflect-101 rows), for t = R..1 then the centre:
//    S = p(y+t) + p(y-t), D = p(y+t) - p(y-t) (exact);  Vg = fma(g_t, S, Vg);
//    Vc = fma(vc_qt, S, Vc);  Vs = fma(vs_qt, D, Vs);  centre: the same fmas with p(y) (vs_q0 = 0).
//  H pass (along each row, reflect-101 columns), taps t = -R..R in order, hs(-t) = -hs(t):
//    Dc = fma(g_|t|, Vg, Dc);
//    mu 0 (b = 0):  re = fma(hc_0t, Vg, re);  im = fma(hs_0t, Vg, im)
//    mu 4 (a = 0):  re = fma(g_|t|, Vc, re); im = fma(g_|t|, Vs, im)
//    other mu (horizontal set p): four chains A = fma(hc_pt, Vc, A), C = fma(hc_pt, Vs, C),
//      B = fma(hs_pt, Vs, B), E = fma(hs_pt, Vc, E); then with the sign of a (mu 5, 6: -1)
//      re = A - sgn*B, im = C + sgn*E  (mu and its mirror share the four sums)
//  then re = fma(-c, Dc, re)   (the reference kernel's DC term -c g(x) g(y)).
void gabor_sep_mag(const uint8_t* img, int w, int h, int index, float* mag) {
  const int nu = index / 7, mu = index % 7;
  const ffd_gabor_sep& s = gabor_sep(nu);
  const int R = s.R, p = FFD_GABOR_P[mu], q = FFD_GABOR_Q[mu];
  const float sgn = (float)FFD_GABOR_SGN[mu];
  std::vector<float> Vg((size_t)w * h), Vc((size_t)w * h), Vs((size_t)w * h);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      auto P = [&](int yy) { return (float)img[reflect101(yy, h) * w + x]; };
      float g = 0.f, c = 0.f, sv = 0.f;
      const float* vc = q > 0 ? s.vc[q - 1] : s.g;
      const float* vs = q > 0 ? s.vs[q - 1] : s.g;
      for (int t = R; t >= 1; t--) {
        const float a = P(y + t), b = P(y - t), S = a + b, D = a - b;
        g = std::fmaf(s.g[t], S, g);
        c = std::fmaf(vc[t], S, c);
        sv = std::fmaf(vs[t], D, sv);
      }
      const float p0 = P(y);
      g = std::fmaf(s.g[0], p0, g);
      c = std::fmaf(vc[0], p0, c);
      sv = std::fmaf(vs[0], p0, sv);
      Vg[(size_t)y * w + x] = g;
      Vc[(size_t)y * w + x] = c;   // q = 0: unused
      Vs[(size_t)y * w + x] = sv;  // q = 0: unused
    }
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      float re = 0.f, im = 0.f, dc = 0.f, A = 0.f, B = 0.f, C = 0.f, E = 0.f;
      for (int t = -R; t <= R; t++) {
        const size_t i = (size_t)y * w + reflect101(x + t, w);
        const int at = t < 0 ? -t : t;
        const float gv = Vg[i];
        dc = std::fmaf(s.g[at], gv, dc);
        if (mu == 0) {
          const float hs = t < 0 ? -s.hs[0][at] : s.hs[0][at];
          re = std::fmaf(s.hc[0][at], gv, re);
          im = std::fmaf(hs, gv, im);
        } else if (mu == 4) {
          re = std::fmaf(s.g[at], Vc[i], re);
          im = std::fmaf(s.g[at], Vs[i], im);
        } else {
          const float hc = s.hc[p][at], hs = t < 0 ? -s.hs[p][at] : s.hs[p][at];
          A = std::fmaf(hc, Vc[i], A);
          C = std::fmaf(hc, Vs[i], C);
          B = std::fmaf(hs, Vs[i], B);
          E = std::fmaf(hs, Vc[i], E);
        }
      }
      if (mu != 0 && mu != 4) {
        re = sgn > 0 ? A - B : A + B;
        im = sgn > 0 ? C + E : C - E;
      }
      re = std::fmaf(-s.c, dc, re);
      const float r2 = re * re, i2 = im * im;
      mag[(size_t)y * w + x] = std::sqrt(i2 + r2);
    }
}

// One Gabor magnitude plane (gaborTransform, FeatureChannelFactory.hpp:253-286).
//  * 7x7 kernels (49 taps < OpenCV's dft_filter_size 50): OpenCV's direct
//    Filter2D, row-major taps, s = 0; s += k*p (no FMA) — bit-exact restatement.
//  * >= 9x9 kernels: OpenCV 2.4.9 switches to a DFT (crossCorr) whose rounding
//    cannot be reproduced; the restatement DEFINES the correlation by the exact
//    separable factorisation of the kernel, gabor_sep_mag above.
void gabor_mag(const uint8_t* img, int w, int h, int index, float* mag) {
  const GaborKernel& g = g_gabor[index];
  if (g.width != 7) return gabor_sep_mag(img, w, h, index, mag);
  const int W = 7, R = 3;
  std::vector<int> rx(w + 2 * R), ry(h + 2 * R);
  for (int i = 0; i < w + 2 * R; i++) rx[i] = reflect101(i - R, w);
  for (int i = 0; i < h + 2 * R; i++) ry[i] = reflect101(i - R, h);
  auto P = [&](int y, int x) -> float { return (float)img[ry[y + R] * w + rx[x + R]]; };
  for (int py = 0; py < h; py++)
    for (int px = 0; px < w; px++) {
      float re = 0.f, im = 0.f;
      for (int r = 0; r < W; r++)
        for (int c = 0; c < W; c++) {
          float p = P(py + r - R, px + c - R);
          re = re + g.re[r * W + c] * p;
          im = im + g.im[r * W + c] * p;
        }
      // pow(r,2), pow(i,2), add(i,r), pow(.,0.5) == sqrt
      float r2 = re * re, i2 = im * im;
      mag[py * w + px] = std::sqrt(i2 + r2);
    }
}

// normalize(NORM_MINMAX, 0, 1) then convertTo(CV_8U, 255) (FeatureChannelFactory.hpp:271-276).
void quantize(const float* mag, int n, uint8_t* out) {
  float mn = mag[0], mx = mag[0];
  for (int i = 1; i < n; i++) { mn = std::min(mn, mag[i]); mx = std::max(mx, mag[i]); }
  double smin = mn, smax = mx, dmin = 0, dmax = 1;
  double scale = (dmax - dmin) * (smax - smin > DBL_EPSILON ? 1. / (smax - smin) : 0);
  double shift = dmin - smin * scale;
  float sf = (float)scale, hf = (float)shift;
  for (int i = 0; i < n; i++) {
    float v = mag[i] * sf + hf;
    out[i] = sat_u8(cv_round(v * 255.f + 0.f));
  }
}

// Sobel 3x3, CV_8U output (saturated), BORDER_REFLECT_101. dy -> channel 36, dx -> 37.
void sobel(const uint8_t* img, int w, int h, bool dy, uint8_t* out) {
  auto I = [&](int y, int x) { return (int)img[reflect101(y, h) * w + reflect101(x, w)]; };
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int v;
      if (dy)
        v = (I(y + 1, x - 1) + 2 * I(y + 1, x) + I(y + 1, x + 1)) - (I(y - 1, x - 1) + 2 * I(y - 1, x) + I(y - 1, x + 1));
      else
        v = (I(y - 1, x + 1) + 2 * I(y, x + 1) + I(y + 1, x + 1)) - (I(y - 1, x - 1) + 2 * I(y, x - 1) + I(y + 1, x - 1));
      out[y * w + x] = sat_u8(v);
    }
}

constexpr int NCH = 38;

// ImageSample(img, {0,1,2}, true) -> 38 integral channels (ImageSample.cpp:77-90).
void extract_channels(const uint8_t* face, int w, int h, uint32_t* ch, int threads) {
  size_t plane = (size_t)(w + 1) * (h + 1);
  integral(face, w, h, ch);  // FC_GRAY
  init_gabor();
  run_pool(threads, 35, [&](int i) {  // FC_GABOR: 35 tasks
    std::vector<float> mag((size_t)w * h);
    std::vector<uint8_t> q((size_t)w * h);
    gabor_mag(face, w, h, i, mag.data());
    quantize(mag.data(), w * h, q.data());
    integral(q.data(), w, h, ch + plane * (1 + i));
  });
  std::vector<uint8_t> s((size_t)w * h);  // FC_SOBEL
  sobel(face, w, h, true, s.data());
  integral(s.data(), w, h, ch + plane * 36);
  sobel(face, w, h, false, s.data());
  integral(s.data(), w, h, ch + plane * 37);
}

// ImageSample::evalTest integral branch (ImageSample.cpp:48-63).
inline int eval_test(const uint32_t* ch, int w, int h, const Node& nd, int px, int py) {
  int W1 = w + 1;
  const uint32_t* I = ch + (size_t)nd.ch * (W1) * (h + 1);
  auto at = [&](int y, int x) { return (int)(float)I[y * W1 + x]; };
  int x1 = px + nd.r1[0], y1 = py + nd.r1[1], w1 = nd.r1[2], h1 = nd.r1[3];
  int x2 = px + nd.r2[0], y2 = py + nd.r2[1], w2 = nd.r2[2], h2 = nd.r2[3];
  int a = at(y1, x1), b = at(y1, x1 + w1), c = at(y1 + h1, x1), d = at(y1 + h1, x1 + w1);
  int p1 = (int)((float)(d - b - c + a) / (float)(w1 * h1));
  a = at(y2, x2); b = at(y2, x2 + w2); c = at(y2 + h2, x2); d = at(y2 + h2, x2 + w2);
  int p2 = (int)((float)(d - b - c + a) / (float)(w2 * h2));
  return p1 - p2;
}

// Tree<S>::evaluateMT (Tree.hpp:173-191): eval true (test <= threshold) -> left.
int walk(const Forest& F, int root, const uint32_t* ch, int w, int h, int px, int py) {
  int i = root;
  while (F.nodes[i].leaf < 0) {
    const Node& nd = F.nodes[i];
    i = (eval_test(ch, w, h, nd, px, py) <= nd.thr) ? nd.left : nd.right;
  }
  return F.nodes[i].leaf;
}

// areaUnderCurve (face_utils.cpp:304-323) with exp := ffd_exp (ffd_numerics.h).
double area_under_curve(float x1, float x2, double mean, double std_) {
  double sum = 0, step = 0.01, t;
  for (double x = x1; x < x2; x += step) {
    t = (x - mean) / std_;
    sum += ffd_exp(-0.5 * (t * t)) * step;
  }
  const double sqrt_2pi = 2.5066282746310002;  // sqrt(2 * M_PI), constant-folded
  return sum * 1.0 / (std_ * sqrt_2pi);
}

inline int to_int_trunc(float v) {  // static_cast<int>(float) on x86-64 (cvttss2si)
  if (!(v > -2147483649.0f && v < 2147483648.0f)) return INT_MIN;
  return (int)v;
}

struct Geometry { int W, H, patch, nhx, nhy, nmx, nmy; float scale; };

// The estimator options (HeadPoseEstimatorOption / MultiPartEstimatorOption, FaceForest.hpp:34-58,
// defaults as their constructors; MeanShiftOption, MeanShift.hpp:16-25).  The FFD y step may differ
// only for SURVEY.md's C4 stress grid; the MeanShift option of analyzeFace is the engine's extension
// (the reference always shifts with a default MeanShiftOption, FaceForest.cpp:89-92).
oracle_options g_opt = {5, 4, 0.5f, 10, 3, 3, 2, 0.5f, 0.25f, 25.f, 10, 7, 0.05f};
#define g_hp_step g_opt.hp_step
#define g_mp_step_x g_opt.mp_step_x
#define g_mp_step_y g_opt.mp_step_y

bool geometry(int bw, int bh, Geometry& g) {
  if (bw <= 0 || bh <= 0) return false;
  // FaceForest.cpp:202-204: scale = 125.f/cols; Size(cols*scale, rows*scale) truncates
  g.scale = (float)g_hp.face_size / (float)bw;
  g.W = (int)((float)bw * g.scale);
  g.H = (int)((float)bh * g.scale);
  g.patch = (int)std::round(g_hp.face_size * g_hp.patch_ratio);  // getPatchSize (Constants.hpp:27-30)
  auto cnt = [](int extent, int patch, int step) { int n = 0; for (int x = 0; x < extent - patch; x += step) n++; return n; };
  g.nhx = cnt(g.W, g.patch, g_hp_step); g.nhy = cnt(g.H, g.patch, g_hp_step);
  g.nmx = cnt(g.W, g.patch, g_mp_step_x); g.nmy = cnt(g.H, g.patch, g_mp_step_y);
  return g.W > 0 && g.H > 0;
}

}  // namespace

// getHeadPoseVotesMT (face_utils.cpp:183-242): patches over the region (x from rx while
// x < rx + rw - patch, step 4, x outer / y inner), every tree per patch, leaf filter fg > 0.5,
// sequential float sums in that order; FaceForest::estimateHeadPose (FaceForest.cpp:60-72).
void estimate_headpose(const uint32_t* ch, int W, int H, int rx, int ry, int rw, int rh, int threads, float* out_mean,
                       float* out_var, std::vector<int>& hp_leafs) {
  const int P = (int)std::round(g_hp.face_size * g_hp.patch_ratio);
  const int HT = (int)g_hp.roots.size();
  std::vector<std::pair<int, int>> hp_patches;
  for (int x = rx; x < rx + rw - P; x += g_hp_step)
    for (int y = ry; y < ry + rh - P; y += g_hp_step) hp_patches.push_back({x, y});
  hp_leafs.assign(hp_patches.size() * HT, 0);
  run_pool(threads, (int)hp_patches.size(), [&](int i) {
    for (int t = 0; t < HT; t++)
      hp_leafs[i * HT + t] = walk(g_hp, g_hp.roots[t], ch, W, H, hp_patches[i].first, hp_patches[i].second);
  });
  float n = 0, sum = 0, sum_sq = 0;
  for (size_t i = 0; i < hp_leafs.size(); ++i) {
    int L = hp_leafs[i];
    if (g_hp.hp_fg[L] > g_opt.hp_min_fg) {  // HeadPoseEstimatorOption::min_foreground_probability
      float m = 0;
      for (int j = 0; j < std::min(g_opt.hp_num_labels, FFD_NUM_HP_LABELS); j++) m += g_hp.hp_labels[L * 5 + j] * j;
      m /= (g_hp.hp_n[L] * g_hp.hp_fg[L]);
      sum += m;
      sum_sq += m * m;
      n++;
    }
  }
  float mean = sum / n;
  float var = (sum_sq / n) - (mean * mean);
  mean -= 2;
  var *= 0.05f;  // NORM_HEADPOSE_VARIANCE_FACTOR (Constants.hpp:67)
  *out_mean = mean;
  *out_var = var;
}

struct MsVote { int x, y; float w; };

// MeanShift::shift (MeanShift.hpp:41-135): getMean, then up to `iters` getWeightedMean passes with the
// kernel exp(-d / lamda) until the mode moves less than `stop`; sequential float sums in list order.
void ms_shift(const MsVote* V, int n, int kernel, int iters, float stop, float& out_x, float& out_y) {
  float mx = 0, my = 0, sw = 0;
  for (int k = 0; k < n; k++) { const MsVote& v = V[k]; float w = v.w; mx += v.x * w; my += v.y * w; sw += w; }
  if (sw > 0) { mx /= sw; my /= sw; }
  bool conv = false;
  const float lamda = (float)kernel;
  for (int it = 0; it < iters && !conv; it++) {
    float sx = 0, sy = 0, s = 0;
    for (int k = 0; k < n; k++) {
      const MsVote& v = V[k];
      float dx = mx - (float)v.x, dy = my - (float)v.y;
      float d = (float)std::sqrt((double)dx * dx + (double)dy * dy);
      d = ffd_expf(-d / lamda);
      float w = v.w * d;
      sx += v.x * w; sy += v.y * w; s += w;
    }
    if (s > 0) { sx /= s; sy /= s; }
    float ddx = sx - mx, ddy = sy - my;
    if (std::sqrt((double)ddx * ddx + (double)ddy * ddy) < stop) conv = true;
    mx = sx; my = sy;
  }
  out_x = mx;
  out_y = my;
}

// getFacialFeaturesVotesMT (face_utils.cpp:244-302) over the region with the given trees, then
// MeanShift::shift per part (MeanShift.hpp:41-135; kernel `ms_kernel`, `ms_iter` iterations, stop
// `ms_stop`: 10 / 7 / 0.05 as FaceForest::estimateFacialFeatures, FaceForest.cpp:74-95): pts = cvRound
// of the modes, in sample coordinates.  Parts >= num_parts (the reference's vectors are num_parts long)
// are reported as (0, 0) with no votes.
void estimate_facial_features(const uint32_t* ch, int W, int H, int rx, int ry, int rw, int rh,
                              const std::vector<int>& trees, int threads, int pts[][2], float* ms_mean,
                              int* vote_counts, std::vector<int>& mp_leafs, int ms_kernel = 10, int ms_iter = 7,
                              float ms_stop = 0.05f) {
  const int NP = std::max(0, std::min(g_opt.mp_num_parts, FFD_NUM_PARTS));
  const int P = (int)std::round(g_hp.face_size * g_hp.patch_ratio);
  const int MT = (int)trees.size();
  std::vector<std::pair<int, int>> mp_patches;
  for (int x = rx; x < rx + rw - P; x += g_mp_step_x)
    for (int y = ry; y < ry + rh - P; y += g_mp_step_y) mp_patches.push_back({x, y});
  mp_leafs.assign(mp_patches.size() * MT, 0);
  run_pool(threads, (int)mp_patches.size(), [&](int i) {
    for (int t = 0; t < MT; t++)
      mp_leafs[i * MT + t] = walk(g_mp, g_mp.roots[trees[t]], ch, W, H, mp_patches[i].first, mp_patches[i].second);
  });
  std::vector<std::vector<MsVote>> votes(FFD_NUM_PARTS);
  for (size_t k = 0; k < mp_leafs.size(); k++) {
    int L = mp_leafs[k];
    int ox = mp_patches[k / MT].first + P / 2, oy = mp_patches[k / MT].second + P / 2;
    for (int i = 0; i < NP; i++) {
      float min_pf = g_opt.mp_min_pf;   // MultiPartEstimatorOption::min_pf
      if (i == 0 || i == 7) min_pf *= 1.5;
      if (g_mp.mp_fg[L] > g_opt.mp_min_fg && g_mp.mp_pf[L * 10 + i] > min_pf && g_mp.mp_var[L * 10 + i] < g_opt.mp_max_var &&
          g_mp.mp_n[L] > g_opt.mp_min_samples)
        votes[i].push_back({g_mp.mp_off[(L * 10 + i) * 2] + ox, g_mp.mp_off[(L * 10 + i) * 2 + 1] + oy, g_mp.mp_fg[L]});
    }
  }
  for (int i = 0; i < FFD_NUM_PARTS; i++) {
    const auto& V = votes[i];
    vote_counts[i] = (int)V.size();
    float mx, my;
    ms_shift(V.data(), (int)V.size(), ms_kernel, ms_iter, ms_stop, mx, my);
    ms_mean[2 * i] = mx;
    ms_mean[2 * i + 1] = my;
    pts[i][0] = i < NP ? cv_round(mx) : 0;
    pts[i][1] = i < NP ? cv_round(my) : 0;
  }
}

// ------------------------------------------------------------------- C API --

namespace {

// ------------------------------------------------- Haar face detector (§8f #1) ----
// FaceForest::detectFace (src/FaceForest.cpp:136-159): CascadeClassifier::detectMultiScale(img,
// boxes, 1.3, 1, 0, Size(30, 30)) on the BGR frame, then the 5 % / 15 % widening clipped to the
// image.  data/haarcascade_frontalface_alt.xml is a new-format (BOOST / HAAR, stump) cascade, so
// OpenCV 2.4.9 runs the image-pyramid path of objdetect/cascadedetect.cpp, restated here:
//   detectMultiScale     factor *= scaleFactor (double); window cvRound(20 f); scaled image
//                        cvRound(cols / f) x cvRound(rows / f) by resize(INTER_LINEAR); scan region
//                        scaled - 20; stop when empty or the window exceeds the image; skip windows
//                        under minSize; yStep = f > 2 ? 1 : 2
//   CascadeClassifierInvoker  x, y over the scan region in steps of yStep; result == 0 (rejected by
//                        stage 0) skips the next x; result > 0 adds Rect(cvRound(x f), cvRound(y f),
//                        window); candidates kept in scan order (OpenCV's strips run in parallel, so
//                        its order is the serial one only without a thread pool; the grouped boxes
//                        do not depend on it except for their output order)
//   HaarEvaluator::setImage / setWindow  integral sum (int) + sqsum (double) of the scaled image;
//                        normrect (1, 1, 18, 18); nf = 324 sqsum - sum^2 (double), sqrt if > 0 else 1,
//                        varianceNormFactor = 1 / nf
//   Feature::calc        float: w0 * S0 + w1 * S1 (+ w2 * S2 when w2 != 0); value = (double)calc * vnf (double)
//   predictOrderedStump  sum (double) += leaf[value < thr ? 0 : 1]; stage fails if sum < (float)stage
//                        threshold - 1e-5f (Data::read THRESHOLD_EPS); returns -stage or 1
//   groupRectangles      (objdetect/cascadedetect.cpp) partition by SimilarRects(0.2), classes with
//                        more than min_neighbors members, averaged with float 1/n and cvRound,
//                        small-inside-large filter; min_neighbors 0 keeps the raw candidates.
// PARITY UNPINNED: OpenCV is not in this image and the reference ships no detections; this is the
// spec the GPU detector (face_alignment_cvpr_2012_amd/csrc/ffd_haar.hip) reproduces bit for bit.
struct Haar {
  int ww = 0, wh = 0;
  std::vector<int32_t> stage_first, stage_ntrees, weak_feature, rect;
  std::vector<float> stage_thr, weak_thr, leaves, weight;
};
Haar g_haar;
bool g_have_haar = false;

void load_haar(const std::map<std::string, Arr>& m) {
  g_have_haar = m.count("haar.window") != 0;
  if (!g_have_haar) return;
  auto vi = [&](const char* k) { const Arr& a = m.at(k); return std::vector<int32_t>(a.p<int32_t>(), a.p<int32_t>() + a.n()); };
  auto vf = [&](const char* k) { const Arr& a = m.at(k); return std::vector<float>(a.p<float>(), a.p<float>() + a.n()); };
  std::vector<int32_t> win = vi("haar.window");
  g_haar.ww = win[0];
  g_haar.wh = win[1];
  g_haar.stage_first = vi("haar.stage_first");
  g_haar.stage_ntrees = vi("haar.stage_ntrees");
  g_haar.stage_thr = vf("haar.stage_threshold");
  for (float& t : g_haar.stage_thr) t = t - 1e-5f;  // Data::read: (float)stageThreshold - THRESHOLD_EPS
  g_haar.weak_feature = vi("haar.weak_feature");
  g_haar.weak_thr = vf("haar.weak_threshold");
  g_haar.leaves = vf("haar.weak_leaves");
  g_haar.rect = vi("haar.feature_rect");
  g_haar.weight = vf("haar.feature_weight");
}

struct IRect { int x, y, w, h; };

// predictOrderedStump at (x, y) of the scaled image's integrals (pitch P = sW + 1)
int haar_run_at(const int32_t* sum, const double* sq, int P, int x, int y) {
  const Haar& H = g_haar;
  const int o = y * P + x;
  // normrect (1, 1, ww - 2, wh - 2)
  const int a = P + 1, b = P + 1 + (H.ww - 2), c = (1 + H.wh - 2) * P + 1, d = c + (H.ww - 2);
  const int valsum = sum[o + a] - sum[o + b] - sum[o + c] + sum[o + d];
  const double valsq = sq[o + a] - sq[o + b] - sq[o + c] + sq[o + d];
  double nf = (double)((H.ww - 2) * (H.wh - 2)) * valsq - (double)valsum * valsum;
  nf = nf > 0. ? std::sqrt(nf) : 1.;
  const double vnf = 1. / nf;
  for (size_t s = 0; s < H.stage_first.size(); s++) {
    double acc = 0.0;
    for (int i = H.stage_first[s], e = i + H.stage_ntrees[s]; i < e; i++) {
      const int f = H.weak_feature[i];
      const int32_t* r = &H.rect[f * 12];
      const float* w = &H.weight[f * 3];
      auto S = [&](int k) {
        const int rx = r[4 * k], ry = r[4 * k + 1], rw = r[4 * k + 2], rh = r[4 * k + 3];
        const int p0 = ry * P + rx, p1 = p0 + rw, p2 = (ry + rh) * P + rx, p3 = p2 + rw;
        return sum[o + p0] - sum[o + p1] - sum[o + p2] + sum[o + p3];
      };
      float ret = w[0] * (float)S(0) + w[1] * (float)S(1);
      if (w[2] != 0.0f) ret += w[2] * (float)S(2);
      // HaarEvaluator::operator() returns double (float calc() * double varianceNormFactor), and
      // predictOrderedStump compares that double with the stump's float threshold
      const double value = (double)ret * vnf;
      acc += (double)H.leaves[2 * i + (value < (double)H.weak_thr[i] ? 0 : 1)];
    }
    if (acc < (double)H.stage_thr[s]) return -(int)s;
  }
  return 1;
}

void haar_scan(const uint8_t* gray, int W, int Hh, double scale_factor, int min_w, int min_h,
               std::vector<IRect>& cand) {
  const Haar& H = g_haar;
  std::vector<uint8_t> scaled;
  std::vector<int32_t> sum;
  std::vector<double> sq;
  for (double factor = 1;; factor *= scale_factor) {
    const int winW = cv_round_d(H.ww * factor), winH = cv_round_d(H.wh * factor);
    const int sW = cv_round_d(W / factor), sH = cv_round_d(Hh / factor);
    const int pW = sW - H.ww, pH = sH - H.wh;
    if (pW <= 0 || pH <= 0) break;
    if (winW > W || winH > Hh) break;  // maxObjectSize defaults to the image size
    if (winW < min_w || winH < min_h) continue;
    scaled.resize((size_t)sW * sH);
    cv_resize(gray, W, Hh, W, scaled.data(), sW, sH);
    const int P = sW + 1;
    sum.assign((size_t)P * (sH + 1), 0);
    sq.assign((size_t)P * (sH + 1), 0.0);
    for (int y = 0; y < sH; y++) {
      int32_t rs = 0;
      double rq = 0;
      for (int x = 0; x < sW; x++) {
        const int v = scaled[(size_t)y * sW + x];
        rs += v;
        rq += (double)(v * v);
        sum[(size_t)(y + 1) * P + x + 1] = sum[(size_t)y * P + x + 1] + rs;
        sq[(size_t)(y + 1) * P + x + 1] = sq[(size_t)y * P + x + 1] + rq;
      }
    }
    const int ystep = factor > 2. ? 1 : 2;
    for (int y = 0; y < pH; y += ystep)
      for (int x = 0; x < pW; x += ystep) {
        const int result = haar_run_at(sum.data(), sq.data(), P, x, y);
        if (result > 0) cand.push_back({cv_round_d(x * factor), cv_round_d(y * factor), winW, winH});
        if (result == 0) x += ystep;
      }
  }
}

// cv::partition with SimilarRects(eps) (union by rank, path compression) -> labels, class count
int haar_partition(const std::vector<IRect>& v, double eps, std::vector<int>& labels) {
  const int N = (int)v.size();
  std::vector<int> parent(N, -1), rank(N, 0);
  auto similar = [&](const IRect& a, const IRect& b) {
    const double delta = eps * (std::min(a.w, b.w) + std::min(a.h, b.h)) * 0.5;
    return std::abs(a.x - b.x) <= delta && std::abs(a.y - b.y) <= delta &&
           std::abs(a.x + a.w - b.x - b.w) <= delta && std::abs(a.y + a.h - b.y - b.h) <= delta;
  };
  for (int i = 0; i < N; i++) {
    int root = i;
    while (parent[root] >= 0) root = parent[root];
    for (int j = 0; j < N; j++) {
      if (i == j || !similar(v[i], v[j])) continue;
      int root2 = j;
      while (parent[root2] >= 0) root2 = parent[root2];
      if (root2 != root) {
        const int rk = rank[root], rk2 = rank[root2];
        if (rk > rk2) {
          parent[root2] = root;
        } else {
          parent[root] = root2;
          rank[root2] += rk == rk2;
          root = root2;
        }
        int k = j, par;
        while ((par = parent[k]) >= 0) { parent[k] = root; k = par; }
        k = i;
        while ((par = parent[k]) >= 0) { parent[k] = root; k = par; }
      }
    }
  }
  labels.assign(N, 0);
  int nclasses = 0;
  for (int i = 0; i < N; i++) {
    int root = i;
    while (parent[root] >= 0) root = parent[root];
    if (rank[root] >= 0) rank[root] = ~nclasses++;
    labels[i] = ~rank[root];
  }
  return nclasses;
}

// groupRectangles(rectList, groupThreshold, eps) without weights
void haar_group(std::vector<IRect>& rects, int thr, double eps) {
  if (thr <= 0 || rects.empty()) return;
  std::vector<int> labels;
  const int nc = haar_partition(rects, eps, labels);
  std::vector<IRect> rr(nc, IRect{0, 0, 0, 0});
  std::vector<int> rw(nc, 0);
  for (size_t i = 0; i < labels.size(); i++) {
    const int c = labels[i];
    rr[c].x += rects[i].x; rr[c].y += rects[i].y; rr[c].w += rects[i].w; rr[c].h += rects[i].h;
    rw[c]++;
  }
  for (int i = 0; i < nc; i++) {
    const IRect r = rr[i];
    const float s = 1.f / rw[i];
    rr[i] = IRect{cv_round((float)r.x * s), cv_round((float)r.y * s), cv_round((float)r.w * s), cv_round((float)r.h * s)};
  }
  rects.clear();
  for (int i = 0; i < nc; i++) {
    const IRect r1 = rr[i];
    const int n1 = rw[i];
    if (n1 <= thr) continue;
    int j;
    for (j = 0; j < nc; j++) {
      const int n2 = rw[j];
      if (j == i || n2 <= thr) continue;
      const IRect r2 = rr[j];
      const int dx = cv_round_d(r2.w * eps), dy = cv_round_d(r2.h * eps);
      if (r1.x >= r2.x - dx && r1.y >= r2.y - dy && r1.x + r1.w <= r2.x + r2.w + dx &&
          r1.y + r1.h <= r2.y + r2.h + dy && (n2 > std::max(3, n1) || n1 < 3))
        break;
    }
    if (j == nc) rects.push_back(r1);
  }
}

// detectFace's widening (FaceForest.cpp:148-158) and intersect (face_utils.cpp:328-346)
IRect widen_box(const IRect& b, int W, int H) {
  const int ox = (int)(b.w * 0.05), oy = (int)(b.w * 0.15);
  const IRect r1{b.x - ox, b.y, b.w + ox * 2, b.h + oy * 2};
  IRect r;
  r.x = r1.x < 0 ? 0 : r1.x;
  r.y = r1.y < 0 ? 0 : r1.y;
  r.w = (r1.x + r1.w < W ? r1.x + r1.w : W) - r.x;
  r.h = (r1.y + r1.h < H ? r1.y + r1.h : H) - r.y;
  if (r.w <= 0 || r.h <= 0) r = IRect{0, 0, 0, 0};
  return r;
}

}  // namespace

extern "C" {

const char* oracle_last_error(void) { return g_err.c_str(); }

int oracle_set_steps(int32_t hp_step, int32_t mp_step_x, int32_t mp_step_y) {
  if (hp_step <= 0 || mp_step_x <= 0 || mp_step_y <= 0) { g_err = "bad step"; return -1; }
  g_hp_step = hp_step; g_mp_step_x = mp_step_x; g_mp_step_y = mp_step_y;
  return 0;
}

int oracle_set_options(const oracle_options* o) {
  static const oracle_options defaults = {5, 4, 0.5f, 10, 3, 3, 2, 0.5f, 0.25f, 25.f, 10, 7, 0.05f};
  if (!o) { g_opt = defaults; return 0; }
  if (o->hp_step <= 0 || o->mp_step_x <= 0 || o->mp_step_y <= 0 || o->ms_kernel == 0) { g_err = "bad options"; return -1; }
  g_opt = *o;
  return 0;
}

int oracle_get_options(oracle_options* o) {
  if (!o) return -1;
  *o = g_opt;
  return 0;
}

int oracle_load_model(const char* path) {
  std::lock_guard<std::mutex> lk(g_mu);
  try {
    auto m = read_container(path);
    build_forest(m, "hp", g_hp, true);
    build_forest(m, "mp", g_mp, false);
    load_haar(m);
    init_gabor();
    g_loaded = true;
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

int oracle_face_geometry(int32_t bw, int32_t bh, int32_t* fw, int32_t* fh, int32_t* nhp, int32_t* nmp) {
  if (!g_loaded) { g_err = "model not loaded"; return -1; }
  Geometry g;
  if (!geometry(bw, bh, g)) { g_err = "degenerate box"; return -1; }
  *fw = g.W; *fh = g.H; *nhp = g.nhx * g.nhy; *nmp = g.nmx * g.nmy;
  return 0;
}

int oracle_detect_faces(const uint8_t* bgr, int32_t w, int32_t h, int32_t stride, int32_t min_size,
                        int32_t min_neighbors, float scale_factor, int32_t widen, int32_t* boxes, int32_t cap,
                        int32_t* n_boxes, int32_t* raw, int32_t raw_cap, int32_t* n_raw) {
  if (!g_loaded || !g_have_haar) { g_err = "model with a Haar cascade not loaded"; return -1; }
  if (!bgr || w <= 0 || h <= 0 || stride < 3 * w || !(scale_factor > 1.f) || !n_boxes) { g_err = "bad arguments"; return -1; }
  std::vector<uint8_t> gray((size_t)w * h);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) gray[(size_t)y * w + x] = gray_px(bgr + (size_t)y * stride + 3 * x);
  std::vector<IRect> cand;
  haar_scan(gray.data(), w, h, (double)scale_factor, min_size, min_size, cand);
  if (n_raw) *n_raw = (int32_t)cand.size();
  for (int i = 0; raw && i < (int)cand.size() && i < raw_cap; i++) {
    raw[4 * i] = cand[i].x; raw[4 * i + 1] = cand[i].y; raw[4 * i + 2] = cand[i].w; raw[4 * i + 3] = cand[i].h;
  }
  haar_group(cand, min_neighbors, 0.2);  // detectMultiScale: GROUP_EPS 0.2
  *n_boxes = (int32_t)cand.size();
  for (int i = 0; boxes && i < (int)cand.size() && i < cap; i++) {
    const IRect r = widen ? widen_box(cand[i], w, h) : cand[i];
    boxes[4 * i] = r.x; boxes[4 * i + 1] = r.y; boxes[4 * i + 2] = r.w; boxes[4 * i + 3] = r.h;
  }
  return 0;
}

int oracle_bgr2gray(const uint8_t* bgr, int32_t w, int32_t h, int32_t stride, uint8_t* gray) {
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) gray[y * w + x] = gray_px(bgr + y * stride + 3 * x);
  return 0;
}

int oracle_resize(const uint8_t* src, int32_t sw, int32_t sh, int32_t sstride, int32_t dw, int32_t dh, uint8_t* dst) {
  cv_resize(src, sw, sh, sstride, dst, dw, dh);
  return 0;
}

int oracle_channels(const uint8_t* face, int32_t w, int32_t h, uint32_t* channels) {
  try { extract_channels(face, w, h, channels, 1); return 0; }
  catch (const std::exception& e) { g_err = e.what(); return -1; }
}

int oracle_gabor_kernel(int32_t index, float* re, float* im, int32_t* width) {
  try { init_gabor(); } catch (const std::exception& e) { g_err = e.what(); return -1; }
  if (index < 0 || index >= (int)g_gabor.size()) return -1;
  const auto& g = g_gabor[index];
  *width = g.width;
  if (re) std::memcpy(re, g.re.data(), g.re.size() * 4);
  if (im) std::memcpy(im, g.im.data(), g.im.size() * 4);
  return 0;
}

int oracle_gabor_mag(const uint8_t* face, int32_t w, int32_t h, int32_t index, float* mag) {
  try { init_gabor(); } catch (const std::exception& e) { g_err = e.what(); return -1; }
  gabor_mag(face, w, h, index, mag);
  return 0;
}

double oracle_area_under_curve(float x1, float x2, double mean, double std_) {
  return area_under_curve(x1, x2, mean, std_);
}

void oracle_meanshift(const int32_t* xy, const float* w, int32_t n, int32_t kernel, int32_t iters, float stop,
                      float* mean_xy) {
  std::vector<MsVote> V(n);
  for (int i = 0; i < n; i++) V[i] = MsVote{xy[2 * i], xy[2 * i + 1], w[i]};
  ms_shift(V.data(), n, kernel, iters, stop, mean_xy[0], mean_xy[1]);
}

double oracle_exp(double x) { return ffd_exp(x); }
float oracle_expf(float x) { return ffd_expf(x); }

int oracle_analyze_face(const uint8_t* bgr, int32_t iw, int32_t ih, int32_t stride, int32_t bx, int32_t by,
                        int32_t bw, int32_t bh, int32_t threads, oracle_face* out, oracle_trace* tr) {
  if (!g_loaded) { g_err = "model not loaded"; return -1; }
  if (bx < 0 || by < 0 || bw <= 0 || bh <= 0 || bx + bw > iw || by + bh > ih) {
    g_err = "bbox outside image";  // cv::Mat ROI assertion in the reference
    return -2;
  }
  Geometry g;
  if (!geometry(bw, bh, g)) { g_err = "degenerate box"; return -2; }
  const int W = g.W, H = g.H;
  std::memset(out, 0, sizeof(*out));
  out->face_w = W; out->face_h = H;

  // a2: gray of the ROI (cvtColor is per-pixel, so ROI-only is identical) + resize
  std::vector<uint8_t> roi((size_t)bw * bh), face((size_t)W * H);
  for (int y = 0; y < bh; y++)
    for (int x = 0; x < bw; x++) roi[y * bw + x] = gray_px(bgr + (size_t)(by + y) * stride + 3 * (bx + x));
  cv_resize(roi.data(), bw, bh, bw, face.data(), W, H);
  if (tr && tr->face) std::memcpy(tr->face, face.data(), face.size());

  // a3-a6: channels
  size_t plane = (size_t)(W + 1) * (H + 1);
  std::vector<uint32_t> ch(plane * NCH);
  try { extract_channels(face.data(), W, H, ch.data(), threads); }
  catch (const std::exception& e) { g_err = e.what(); return -1; }
  if (tr && tr->channels) std::memcpy(tr->channels, ch.data(), ch.size() * 4);

  // a13/a14: estimateHeadPose over the whole scaled face (FaceForest.cpp:211)
  float mean = 0, var = 0;
  std::vector<int> hp_leafs;
  estimate_headpose(ch.data(), W, H, 0, 0, W, H, threads, &mean, &var, hp_leafs);
  if (tr && tr->hp_leaves) std::memcpy(tr->hp_leaves, hp_leafs.data(), hp_leafs.size() * 4);
  out->headpose = mean;
  out->pose_variance = var;

  // a15: pose histogram + tree selection (FaceForest.cpp:214-250)
  const int NF = g_mp.n_forests, NT = g_mp.ntrees_per_forest;
  std::vector<float> poseT = {-2.5f, -0.35f, -0.20f, 0.20f, 0.35f, 2.5f};
  std::vector<float> pose_freq(NF);
  float max_area = 0;
  int dominant = 0;
  for (int j = 0; j < NF; j++) {
    float area = (float)area_under_curve(poseT[j], poseT[j + 1], mean, std::sqrt((double)var));
    pose_freq[j] = area;
    if (max_area < area) { max_area = area; dominant = j; }
  }
  if (tr && tr->pose_freq) std::memcpy(tr->pose_freq, pose_freq.data(), NF * 4);
  std::vector<int> trees;
  for (int i = 0; i < NF; i++) {
    int nt = to_int_trunc(std::floor(pose_freq[i] * NT));
    nt = std::min(nt, NT);  // getTree(j >= NT) is out of range in the reference
    for (int j = 0; j < nt && (int)trees.size() < ORACLE_MAX_TREES; j++) trees.push_back(i * NT + j);
  }
  for (int i = (int)trees.size(); i < NT; i++) trees.push_back(dominant * NT + i);
  out->n_trees = (int)trees.size();
  if (tr && tr->trees) std::memcpy(tr->trees, trees.data(), trees.size() * 4);

  // a16-a18: estimateFacialFeatures over the whole scaled face (FaceForest.cpp:253), then the
  // rescale of FaceForest.cpp:255-257
  std::vector<int> mp_leafs;
  int pts[FFD_NUM_PARTS][2];
  float msm[2 * FFD_NUM_PARTS];
  int vc[FFD_NUM_PARTS];
  estimate_facial_features(ch.data(), W, H, 0, 0, W, H, trees, threads, pts, msm, vc, mp_leafs, g_opt.ms_kernel,
                           g_opt.ms_iter, g_opt.ms_stop);
  if (tr && tr->mp_leaves) std::memcpy(tr->mp_leaves, mp_leafs.data(), mp_leafs.size() * 4);
  if (tr && tr->vote_counts) std::memcpy(tr->vote_counts, vc, sizeof(vc));
  if (tr && tr->ms_mean) std::memcpy(tr->ms_mean, msm, sizeof(msm));
  float inv_scale = 1.0f / g.scale;
  for (int i = 0; i < FFD_NUM_PARTS; i++) {
    // FaceForest.cpp:255-257: Point_<int> *= 1.0f/scale -> cvRound(x * inv)
    out->points[i][0] = cv_round((float)pts[i][0] * inv_scale);
    out->points[i][1] = cv_round((float)pts[i][1] * inv_scale);
  }
  return 0;
}

static bool region_ok(int W, int H, int rx, int ry, int rw, int rh) {
  return rx >= 0 && ry >= 0 && rw > 0 && rh > 0 && rx + rw <= W && ry + rh <= H;
}

int oracle_estimate_headpose(const uint32_t* channels, int32_t W, int32_t H, int32_t rx, int32_t ry, int32_t rw,
                             int32_t rh, float* headpose, float* variance) {
  if (!g_loaded) { g_err = "model not loaded"; return -1; }
  if (!region_ok(W, H, rx, ry, rw, rh)) { g_err = "face_bbox outside the image sample"; return -2; }
  std::vector<int> leafs;
  estimate_headpose(channels, W, H, rx, ry, rw, rh, 1, headpose, variance, leafs);
  return 0;
}

int oracle_estimate_facial_features(const uint32_t* channels, int32_t W, int32_t H, int32_t rx, int32_t ry,
                                    int32_t rw, int32_t rh, const int32_t* tree_ids, int32_t n_trees,
                                    int32_t* points) {
  if (!g_loaded) { g_err = "model not loaded"; return -1; }
  if (!region_ok(W, H, rx, ry, rw, rh)) { g_err = "face_bbox outside the image sample"; return -2; }
  std::vector<int> trees(tree_ids, tree_ids + n_trees), leafs;
  int pts[FFD_NUM_PARTS][2], vc[FFD_NUM_PARTS];
  float msm[2 * FFD_NUM_PARTS];
  estimate_facial_features(channels, W, H, rx, ry, rw, rh, trees, 1, pts, msm, vc, leafs);
  for (int i = 0; i < FFD_NUM_PARTS; i++) { points[2 * i] = pts[i][0]; points[2 * i + 1] = pts[i][1]; }
  return 0;
}

// Tree<S>::evaluateMT (Tree.hpp:173-191) for an explicit patch list: leaf[p * n_trees + t] of tree tree_ids[t]
// (kind 0 head pose, 1 FFD global id) from the patch at (xy[2p], xy[2p + 1]).
int oracle_eval_patches(const uint32_t* channels, int32_t W, int32_t H, int32_t kind, const int32_t* xy, int32_t n,
                        const int32_t* tree_ids, int32_t n_trees, int32_t* leaf) {
  if (!g_loaded) { g_err = "model not loaded"; return -1; }
  const Forest& F = kind == 0 ? g_hp : g_mp;
  for (int p = 0; p < n; p++)
    for (int t = 0; t < n_trees; t++)
      leaf[p * n_trees + t] = walk(F, F.roots[tree_ids[t]], channels, W, H, xy[2 * p], xy[2 * p + 1]);
  return 0;
}

}  // extern "C"
