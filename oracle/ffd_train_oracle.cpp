// ffd_train_oracle.cpp — CPU restatement of the reference's tree training: facial-feature
// (Tree<MPSample>) and head-pose (Tree<HeadPoseSample>, below) trees.
//
// TEST INFRASTRUCTURE ONLY: the checker for the HIP training path (csrc/ffd_train.*).  Only tests/
// and tools/ load it; the product library never links or calls it.
//
// Follows (paths relative to /root/reference):
//   src/train_ffd.cpp:66-112          trainTree: rng.seed(idx_tree + 1), npatches random patches per image
//   src/MPSample.cpp:13-41            MPSample training ctor: part offsets, m_prob = expf(-d / lamda), m_is_positive
//   include/ImageSample.hpp:35-81     SimplePatchFeature::generate (9 boost::uniform_int draws)
//   src/ImageSample.cpp:40-47         evalTest, non-integral branch (training samples: use_integral = false)
//   src/MPSample.cpp:86-144           generateSplit, evalSplit (mode = 1: entropie_parts)
//   src/MPSample.cpp:146-248          makeLeaf
//   src/MPSample.cpp:276-297          entropie_parts
//   include/SplitGen.hpp:74-101       generateMT (one mt19937 per stripe), sort by (value, index)
//   include/SplitGen.hpp:103-167      splitSamples (margin 0: lower_bound of the threshold)
//   include/SplitGen.hpp:170-231      findThreshold (25 thresholds uniform in [min, max])
//   include/Tree.hpp:43-63,102-171    Tree ctor, grow (depth-first, left then right)
//   include/Tree.hpp:261-308          findOptimalSplit (first strict maximum over stripes), applyOptimalSplit
//
// Definitions where the reference is not deterministic or depends on its toolchain (parity unpinned:
// the reference needs OpenCV 2.4.9 + Boost 1.55 and LFW, none of which is here):
//   * SplitGen::generateMT seeds each stripe with abs(stripe + 1) * std::time(NULL) (SplitGen.hpp:78);
//     here time(NULL) is  split_seed + the node's heap index (root 1, children 2h and 2h + 1), i.e. a
//     clock that differs per node, and the product (uint32) is the seed as in mt19937(value).
//   * cv::Rect(rand_x(), rand_y(), ...) (train_ffd.cpp:108): argument evaluation order is unspecified in
//     C++; here x is drawn first.
//   * entropie_parts' `p * log(p)` with float p: the C library's double log (ffd_log, include/ffd_numerics.h).
//   * sum /= (float)set.size() (cv::Mat): convertTo with scale (float)(1.0 / n), i.e. sum * scale + 0.
//   * boost::mt19937 == std::mt19937 (same recurrence, tempering and seeding); boost::uniform_int is
//     restated from Boost.Random's generate_uniform_int (bucket division with rejection).
//   * The images are the caller's training ROIs (the gray enlarged face at face_size scale,
//     train_ffd.cpp:82-99) with their landmarks in ROI coordinates; the annotation shuffle and the
//     images-per-class selection (train_ffd.cpp:57-62) are the caller's.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "ffd_numerics.h"
#include "ffd_oracle.h"

namespace {

constexpr int NCH = 38;
constexpr float PATCH_CLOSE_TO_FEATURE = 0.09f;  // Constants.hpp:68

// Boost.Random generate_uniform_int for a 32-bit engine (brange = 2^32 - 1 > range).
int uniform_int(std::mt19937& eng, int lo, int hi) {
  const uint32_t range = (uint32_t)(hi - lo);
  if (range == 0) return lo;  // no draw
  const uint32_t brange = 0xFFFFFFFFu;
  uint32_t bucket = brange / (range + 1u);
  if (brange % (range + 1u) == range) ++bucket;
  for (;;) {
    const uint32_t r = (uint32_t)eng() / bucket;
    if (r <= range) return lo + (int)r;
  }
}

struct Feature {
  int ch;
  int r1[4], r2[4];  // x, y, w, h
};

// SimplePatchFeature::generate(patch_size, rng, 38, 1.0) (ImageSample.hpp:35-81)
Feature generate(int patch_size, std::mt19937& rng) {
  Feature f;
  f.ch = uniform_int(rng, 0, NCH - 1);
  const int sub = (int)(patch_size * 1.0f);
  const int smax = (int)((sub - 1) * 0.75);
  f.r1[2] = uniform_int(rng, 1, smax);
  f.r1[3] = uniform_int(rng, 1, smax);
  f.r2[2] = uniform_int(rng, 1, smax);
  f.r2[3] = uniform_int(rng, 1, smax);
  f.r1[0] = uniform_int(rng, 0, sub - f.r1[2] - 1);
  f.r1[1] = uniform_int(rng, 0, sub - f.r1[3] - 1);
  f.r2[0] = uniform_int(rng, 0, sub - f.r2[2] - 1);
  f.r2[1] = uniform_int(rng, 0, sub - f.r2[3] - 1);
  return f;
}

struct Image {
  int w, h;
  std::vector<uint32_t> ch;  // 38 integral planes (h+1) x (w+1), exact
};

struct Sample {
  int img, x, y;
  int off[10][2];
  float prob[10];
  bool pos;
};

struct Trainer {
  const oracle_train_param* P;
  int np, ps;
  std::vector<Image> imgs;
  std::vector<Sample> samples;
  std::mt19937 tree_rng;
  // output (pre-order)
  std::vector<int32_t> node_leaf;
  std::vector<int16_t> node_split;
  std::vector<double> node_info;
  std::vector<int32_t> leaf_n;
  std::vector<float> leaf_fg, leaf_var, leaf_pf;
  std::vector<int16_t> leaf_off;
  int64_t i_node = 0;

  // ImageSample::evalTest, non-integral branch: (int)(sum / (float)(w h)) = floor(sum / area)
  int eval(const Feature& f, const Sample& s) const {
    const Image& im = imgs[s.img];
    const int W1 = im.w + 1;
    const uint32_t* I = im.ch.data() + (size_t)f.ch * W1 * (im.h + 1);
    auto rect = [&](const int* r) {
      const int x = s.x + r[0], y = s.y + r[1], w = r[2], h = r[3];
      const int64_t S = (int64_t)I[(y + h) * W1 + x + w] - I[y * W1 + x + w] - I[(y + h) * W1 + x] + I[y * W1 + x];
      return (int)((double)S / (double)(float)(w * h));
    };
    return rect(f.r1) - rect(f.r2);
  }

  // entropie_parts (MPSample.cpp:276-297) over samples list[a..b)
  double entropy_parts(const std::vector<int>& order, const std::vector<int>& list, int a, int b) const {
    float sum[10] = {0};
    for (int i = a; i < b; i++) {
      const Sample& s = samples[list[order[i]]];
      for (int p = 0; p < np; p++) sum[p] = sum[p] + s.prob[p];
    }
    const float sf = (float)(1.0 / (double)(float)(b - a));
    double e = 0;
    for (int p = 0; p < np; p++) {
      const float pb = sum[p] * sf + 0.0f;
      if (pb > 0) e += (double)pb * ffd_log((double)pb);
    }
    return e;
  }

  // stable sort of list positions by value (std::sort of (value, index) pairs)
 public:
  static void sort_by_value(const std::vector<int>& vals, std::vector<int>& order) {
    const int n = (int)vals.size();
    int cnt[512] = {0};
    for (int v : vals) cnt[v + 256]++;
    int start[512], acc = 0;
    for (int b = 0; b < 512; b++) { start[b] = acc; acc += cnt[b]; }
    order.assign(n, 0);
    for (int i = 0; i < n; i++) order[start[vals[i] + 256]++] = i;
  }

  void make_leaf(const std::vector<int>& list) {  // MPSample::makeLeaf (MPSample.cpp:146-248)
    const int l = (int)leaf_n.size();
    const int n = (int)list.size();
    leaf_n.push_back(n);
    for (int j = 0; j < 10; j++) {
      leaf_off.push_back(0);
      leaf_off.push_back(0);
      leaf_var.push_back(FLT_MAX);
      leaf_pf.push_back(0.f);
    }
    float fg = 0;
    int size = 0;
    for (int i : list) size += samples[i].pos ? 1 : 0;
    if (size > 0) {
      for (int j = 0; j < np; j++) {
        int mx = 0, my = 0;
        float sum_dist = 0;
        for (int i : list)
          if (samples[i].pos) {
            sum_dist += samples[i].prob[j];
            mx += samples[i].off[j][0];
            my += samples[i].off[j][1];
          }
        mx /= size;
        my /= size;
        leaf_pf[l * 10 + j] = sum_dist / (float)size;
        leaf_off[(l * 10 + j) * 2] = (int16_t)mx;
        leaf_off[(l * 10 + j) * 2 + 1] = (int16_t)my;
        double var = 0.0;
        for (int i : list)
          if (samples[i].pos) {
            const int x = samples[i].off[j][0], y = samples[i].off[j][1];
            const float dist = (float)std::sqrt((double)((x - mx) * (x - mx) + (y - my) * (y - my)));
            var += dist;
          }
        var /= size;
        leaf_var[l * 10 + j] = (float)var;
      }
      fg = size / (float)n;
    }
    leaf_fg.push_back(fg);
    node_leaf.push_back(l);
    for (int j = 0; j < 10; j++) node_split.push_back(0);
    node_info.push_back(0.0);
  }

  void grow(const std::vector<int>& list, int depth, uint32_t heap) {
    const int n = (int)list.size();
    if (n < P->min_patches || depth >= P->max_depth) {
      make_leaf(list);
      i_node += (int64_t)(std::pow(2.0f, (float)(P->max_depth - depth)) - 1);
      return;
    }
    (void)uniform_int(tree_rng, 0, 100);  // rand_split() (Tree.hpp:267-269): MPSample::evalSplit ignores it
    const uint32_t T = P->split_seed + heap;
    Feature best_f{};
    double best_info = -DBL_MAX;
    int best_thr = 0;
    std::vector<int> vals(n), order;
    for (int stripe = 0; stripe < P->ntests; stripe++) {
      std::mt19937 rng((uint32_t)((uint64_t)(stripe + 1) * (uint64_t)T));
      const Feature f = generate(ps, rng);
      for (int i = 0; i < n; i++) vals[i] = eval(f, samples[list[i]]);
      sort_by_value(vals, order);
      double info = -DBL_MAX;
      int thr = 0;
      const int vmin = vals[order.front()], vmax = vals[order.back()], range = vmax - vmin;
      if (range > 0) {
        for (int j = 0; j < P->num_thresholds; j++) {
          const int t = uniform_int(rng, 0, range) + vmin;
          int k = 0;  // lower_bound: samples with value < t
          while (k < n && vals[order[k]] < t) k++;
          if (k < 2 || n - k < 2) continue;
          const double ea = entropy_parts(order, list, 0, k), eb = entropy_parts(order, list, k, n);
          const double v = (ea * (double)k + eb * (double)(n - k)) / (double)n;
          if (v > info) { info = v; thr = t; }
        }
      }
      if (info > best_info) { best_info = info; best_thr = thr; best_f = f; }
    }
    if (best_info == -DBL_MAX) {  // no valid split: leaf (Tree.hpp:156-165)
      make_leaf(list);
      i_node += (int64_t)(std::pow(2.0f, (float)(P->max_depth - depth)) - 1);
      return;
    }
    // applyOptimalSplit: the children are the sorted list split at the threshold
    for (int i = 0; i < n; i++) vals[i] = eval(best_f, samples[list[i]]);
    sort_by_value(vals, order);
    int k = 0;
    while (k < n && vals[order[k]] < best_thr) k++;
    std::vector<int> A(k), B(n - k);
    for (int i = 0; i < k; i++) A[i] = list[order[i]];
    for (int i = k; i < n; i++) B[i - k] = list[order[i]];
    node_leaf.push_back(-1);
    const int16_t s[10] = {(int16_t)best_f.ch, (int16_t)best_f.r1[0], (int16_t)best_f.r1[1], (int16_t)best_f.r1[2],
                           (int16_t)best_f.r1[3], (int16_t)best_f.r2[0], (int16_t)best_f.r2[1], (int16_t)best_f.r2[2],
                           (int16_t)best_f.r2[3], (int16_t)best_thr};
    node_split.insert(node_split.end(), s, s + 10);
    node_info.push_back(best_info);
    i_node++;
    grow(A, depth + 1, 2 * heap);
    grow(B, depth + 1, 2 * heap + 1);
  }
};

// ---------------------------------------------------------------- head pose --
// Tree<HeadPoseSample> training (src/train_headpose.cpp:40-143, src/HeadPoseSample.cpp:30-248).
//   * trainTree's samples: per image (the caller's gray image already scaled so the face box is
//     face_size wide, train_headpose.cpp:83-96), npatches * (1 - 0.2f) positive patches at
//     box.(x, y) + U{0 .. face_size - ps - 1} (label pose + 2), then npatches * 0.2f negative patches
//     at U{0 .. cols - ps - 1} x U{0 .. rows - ps - 1} that miss the face box (intersect(),
//     face_utils.cpp:325-346), up to 100 attempts each (a patch whose 100th attempt is reached is
//     dropped, as the reference's `attempt == max_attempts` test does even when that attempt missed
//     the box); every draw from the tree's mt19937 (seed idx_tree + 1), x before y.
//   * findOptimalSplit draws split_mode = U{0..100} from the TREE's generator once per searched node
//     (Tree.hpp:267-274), so the nodes' modes follow the depth-first order of the search.
//   * evalSplit (HeadPoseSample.cpp:64-87): split_mode < 50 -> size-weighted entropie (the fg / bg
//     entropy, :120-143), else gain2 (the negative variance of the positive labels, :228-248) weighted
//     by the positive counts; both are functions of the class counts of each side.
//   * makeLeaf (:89-118): fg fraction, sample count, histogram of the positive labels.
struct HPSample {
  int img, x, y, label;
};

// HeadPoseSample::entropie (HeadPoseSample.cpp:120-143) over the set's class counts
double hp_entropie(double p, int64_t size) {
  double e = 0;
  const double p_pos = p / (double)size;
  if (p_pos > 0) e += p_pos * ffd_log(p_pos);
  const double p_neg = ((double)size - p) / (double)size;
  if (p_neg > 0) e += p_neg * ffd_log(p_neg);
  return e;
}

// HeadPoseSample::gain2 (HeadPoseSample.cpp:228-248): n positives, label sum and sum of squares
double hp_gain2(double n, double sum, double sq_sum) {
  const double mean = sum / n;
  const double variance = (sq_sum / n) - (mean * mean);
  return -variance;
}

struct HPTrainer {
  const oracle_train_param* P;
  int ps;
  std::vector<Image> imgs;
  std::vector<HPSample> samples;
  std::mt19937 tree_rng;
  std::vector<int32_t> node_leaf;
  std::vector<int16_t> node_split;
  std::vector<double> node_info;
  std::vector<int32_t> leaf_n, leaf_labels, node_mode;
  std::vector<float> leaf_fg;
  int64_t i_node = 0;

  int eval(const Feature& f, const HPSample& s) const {
    const Image& im = imgs[s.img];
    const int W1 = im.w + 1;
    const uint32_t* I = im.ch.data() + (size_t)f.ch * W1 * (im.h + 1);
    auto rect = [&](const int* r) {
      const int x = s.x + r[0], y = s.y + r[1], w = r[2], h = r[3];
      const int64_t S = (int64_t)I[(y + h) * W1 + x + w] - I[y * W1 + x + w] - I[(y + h) * W1 + x] + I[y * W1 + x];
      return (int)((double)S / (double)(float)(w * h));
    };
    return rect(f.r1) - rect(f.r2);
  }

  // evalSplit over the two sets list[order[0..k)], list[order[k..n)], literally: counts by loops
  double eval_split(const std::vector<int>& order, const std::vector<int>& list, int k, int mode) const {
    const int n = (int)order.size();
    auto stats = [&](int a, int b, double& p, double& sum, double& sq) {
      p = 0; sum = 0; sq = 0;
      for (int i = a; i < b; i++) {
        const HPSample& s = samples[list[order[i]]];
        if (s.label >= 0) {
          p += 1;
          sum += s.label;
          sq += s.label * s.label;
        }
      }
    };
    double pa, sa, qa, pb, sb, qb;
    stats(0, k, pa, sa, qa);
    stats(k, n, pb, sb, qb);
    if (mode < 50) {
      const double ea = hp_entropie(pa, k), eb = hp_entropie(pb, n - k);
      return (ea * (double)k + eb * (double)(n - k)) / (double)(k + n - k);
    }
    const int size_a = (int)pa, size_b = (int)pb;
    const double ga = hp_gain2(pa, sa, qa), gb = hp_gain2(pb, sb, qb);
    return (ga * size_a + gb * size_b) / (double)(size_b + size_a);
  }

  void make_leaf(const std::vector<int>& list) {
    const int l = (int)leaf_n.size();
    const int n = (int)list.size();
    int size = 0;
    for (int i : list) size += samples[i].label >= 0 ? 1 : 0;
    leaf_n.push_back(n);
    leaf_fg.push_back((float)size / (float)n);
    for (int j = 0; j < 5; j++) leaf_labels.push_back(0);
    if (size > 0)
      for (int i : list)
        if (samples[i].label >= 0) leaf_labels[l * 5 + samples[i].label]++;
    node_leaf.push_back(l);
    for (int j = 0; j < 10; j++) node_split.push_back(0);
    node_info.push_back(0.0);
    node_mode.push_back(-1);
  }

  void grow(const std::vector<int>& list, int depth, uint32_t heap) {
    const int n = (int)list.size();
    if (n < P->min_patches || depth >= P->max_depth) {
      make_leaf(list);
      i_node += (int64_t)(std::pow(2.0f, (float)(P->max_depth - depth)) - 1);
      return;
    }
    const int mode = uniform_int(tree_rng, 0, 100);  // rand_split() (Tree.hpp:267-274)
    const uint32_t T = P->split_seed + heap;
    Feature best_f{};
    double best_info = -DBL_MAX;
    int best_thr = 0;
    std::vector<int> vals(n), order;
    for (int stripe = 0; stripe < P->ntests; stripe++) {
      std::mt19937 rng((uint32_t)((uint64_t)(stripe + 1) * (uint64_t)T));
      const Feature f = generate(ps, rng);
      for (int i = 0; i < n; i++) vals[i] = eval(f, samples[list[i]]);
      Trainer::sort_by_value(vals, order);
      double info = -DBL_MAX;
      int thr = 0;
      const int vmin = vals[order.front()], vmax = vals[order.back()], range = vmax - vmin;
      if (range > 0) {
        for (int j = 0; j < P->num_thresholds; j++) {
          const int t = uniform_int(rng, 0, range) + vmin;
          int k = 0;
          while (k < n && vals[order[k]] < t) k++;
          if (k < 2 || n - k < 2) continue;
          const double v = eval_split(order, list, k, mode);
          if (v > info) { info = v; thr = t; }
        }
      }
      if (info > best_info) { best_info = info; best_thr = thr; best_f = f; }
    }
    if (best_info == -DBL_MAX) {
      make_leaf(list);
      i_node += (int64_t)(std::pow(2.0f, (float)(P->max_depth - depth)) - 1);
      return;
    }
    for (int i = 0; i < n; i++) vals[i] = eval(best_f, samples[list[i]]);
    Trainer::sort_by_value(vals, order);
    int k = 0;
    while (k < n && vals[order[k]] < best_thr) k++;
    std::vector<int> A(k), B(n - k);
    for (int i = 0; i < k; i++) A[i] = list[order[i]];
    for (int i = k; i < n; i++) B[i - k] = list[order[i]];
    node_leaf.push_back(-1);
    const int16_t s[10] = {(int16_t)best_f.ch, (int16_t)best_f.r1[0], (int16_t)best_f.r1[1], (int16_t)best_f.r1[2],
                           (int16_t)best_f.r1[3], (int16_t)best_f.r2[0], (int16_t)best_f.r2[1], (int16_t)best_f.r2[2],
                           (int16_t)best_f.r2[3], (int16_t)best_thr};
    node_split.insert(node_split.end(), s, s + 10);
    node_info.push_back(best_info);
    node_mode.push_back(mode);
    i_node++;
    grow(A, depth + 1, 2 * heap);
    grow(B, depth + 1, 2 * heap + 1);
  }
};

// intersect (face_utils.cpp:325-346) is empty
bool hp_disjoint(int ax, int ay, int aw, int ah, int bx, int by, int bw, int bh) {
  const int x = ax < bx ? bx : ax, y = ay < by ? by : ay;
  const int w = (ax + aw < bx + bw ? ax + aw : bx + bw) - x, h = (ay + ah < by + bh ? ay + ah : by + bh) - y;
  return w <= 0 || h <= 0;
}

std::string g_err;

}  // namespace

struct oracle_train_tree {
  Trainer t;
};

extern "C" {

int oracle_train_mp_tree(const uint8_t* const* images, const int32_t* widths, const int32_t* heights,
                         const int32_t* parts, int32_t n_images, int32_t n_parts, const oracle_train_param* p,
                         oracle_train_tree** out) {
  try {
    if (!images || !widths || !heights || !parts || !p || !out || n_images <= 0 || n_parts < 1 || n_parts > 10)
      throw std::runtime_error("bad arguments");
    auto* h = new oracle_train_tree;
    Trainer& T = h->t;
    T.P = p;
    T.np = n_parts;
    T.ps = (int)std::round(p->face_size * p->patch_size_ratio);  // ForestParam::getPatchSize
    T.tree_rng.seed(p->tree_seed);
    T.imgs.resize(n_images);
    for (int i = 0; i < n_images; i++) {
      Image& im = T.imgs[i];
      im.w = widths[i];
      im.h = heights[i];
      if (im.w < T.ps + 4 || im.h < T.ps + 4) throw std::runtime_error("image smaller than a patch");
      im.ch.resize((size_t)NCH * (im.w + 1) * (im.h + 1));
      if (oracle_channels(images[i], im.w, im.h, im.ch.data()) != 0) throw std::runtime_error("channels failed");
      // patches (train_ffd.cpp:102-111): x in [1, cols - ps - 2], y in [1, rows - ps - 2], x drawn first
      for (int j = 0; j < p->npatches; j++) {
        Sample s;
        s.img = i;
        s.x = uniform_int(T.tree_rng, 1, im.w - T.ps - 2);
        s.y = uniform_int(T.tree_rng, 1, im.h - T.ps - 2);
        // MPSample ctor (MPSample.cpp:13-41)
        const int cx = s.x + T.ps / 2, cy = s.y + T.ps / 2;
        s.pos = false;
        for (int k = 0; k < 10; k++) {
          s.off[k][0] = s.off[k][1] = 0;
          s.prob[k] = 0.f;
        }
        for (int k = 0; k < n_parts; k++) {
          s.off[k][0] = parts[(i * n_parts + k) * 2] - cx;
          s.off[k][1] = parts[(i * n_parts + k) * 2 + 1] - cy;
          const float fx = (float)s.off[k][0] / (float)p->face_size, fy = (float)s.off[k][1] / (float)p->face_size;
          const float d = (float)std::sqrt((double)fx * fx + (double)fy * fy);
          s.prob[k] = ffd_expf(-d / p->lamda);
          if (s.prob[k] > PATCH_CLOSE_TO_FEATURE) s.pos = true;
        }
        T.samples.push_back(s);
      }
    }
    std::vector<int> all(T.samples.size());
    for (size_t i = 0; i < all.size(); i++) all[i] = (int)i;
    T.grow(all, 0, 1u);
    *out = h;
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

int oracle_train_tree_size(const oracle_train_tree* h, int64_t* n_nodes, int64_t* n_leaves, int64_t* i_node) {
  if (!h) return -1;
  if (n_nodes) *n_nodes = (int64_t)h->t.node_leaf.size();
  if (n_leaves) *n_leaves = (int64_t)h->t.leaf_n.size();
  if (i_node) *i_node = h->t.i_node;
  return 0;
}

int oracle_train_tree_get(const oracle_train_tree* h, int32_t* node_leaf, int16_t* node_split, double* node_info,
                          int32_t* leaf_n, float* leaf_fg, int16_t* leaf_offset, float* leaf_var, float* leaf_pf,
                          int32_t* samples_xy) {
  if (!h) return -1;
  const Trainer& t = h->t;
  auto cp = [](auto* dst, const auto& v) {
    if (dst && !v.empty()) std::memcpy(dst, v.data(), v.size() * sizeof(v[0]));
  };
  cp(node_leaf, t.node_leaf);
  cp(node_split, t.node_split);
  cp(node_info, t.node_info);
  cp(leaf_n, t.leaf_n);
  cp(leaf_fg, t.leaf_fg);
  cp(leaf_offset, t.leaf_off);
  cp(leaf_var, t.leaf_var);
  cp(leaf_pf, t.leaf_pf);
  if (samples_xy)
    for (size_t i = 0; i < t.samples.size(); i++) {
      samples_xy[3 * i] = t.samples[i].img;
      samples_xy[3 * i + 1] = t.samples[i].x;
      samples_xy[3 * i + 2] = t.samples[i].y;
    }
  return 0;
}

void oracle_train_tree_free(oracle_train_tree* h) { delete h; }

struct oracle_hp_tree {
  HPTrainer t;
};

int oracle_train_hp_tree(const uint8_t* const* images, const int32_t* widths, const int32_t* heights,
                         const int32_t* faces, const int32_t* poses, int32_t n_images, const oracle_train_param* p,
                         oracle_hp_tree** out) {
  try {
    if (!images || !widths || !heights || !faces || !poses || !p || !out || n_images <= 0)
      throw std::runtime_error("bad arguments");
    auto* h = new oracle_hp_tree;
    HPTrainer& T = h->t;
    T.P = p;
    T.ps = (int)std::round(p->face_size * p->patch_size_ratio);
    T.tree_rng.seed(p->tree_seed);
    T.imgs.resize(n_images);
    const int npos_hi = 0;
    (void)npos_hi;
    for (int i = 0; i < n_images; i++) {
      Image& im = T.imgs[i];
      im.w = widths[i];
      im.h = heights[i];
      const int* b = faces + 4 * i;
      if (im.w < T.ps + 1 || im.h < T.ps + 1 || b[0] < 0 || b[1] < 0 || b[0] + p->face_size - 1 > im.w ||
          b[1] + p->face_size - 1 > im.h || poses[i] < -2 || poses[i] > 2)
        throw std::runtime_error("image " + std::to_string(i) + ": face box or size out of range");
      im.ch.resize((size_t)NCH * (im.w + 1) * (im.h + 1));
      if (oracle_channels(images[i], im.w, im.h, im.ch.data()) != 0) throw std::runtime_error("channels failed");
      // positives (train_headpose.cpp:101-109)
      for (int j = 0; j < p->npatches * (1 - 0.2f); j++) {
        HPSample s;
        s.img = i;
        s.x = b[0] + uniform_int(T.tree_rng, 0, p->face_size - T.ps - 1);
        s.y = b[1] + uniform_int(T.tree_rng, 0, p->face_size - T.ps - 1);
        s.label = poses[i] + 2;
        T.samples.push_back(s);
      }
      // negatives (train_headpose.cpp:111-127)
      for (int j = 0; j < p->npatches * 0.2f; j++) {
        int x, y, attempt = 0;
        bool miss;
        do {
          x = uniform_int(T.tree_rng, 0, im.w - T.ps - 1);
          y = uniform_int(T.tree_rng, 0, im.h - T.ps - 1);
          miss = hp_disjoint(x, y, T.ps, T.ps, b[0], b[1], b[2], b[3]);
          attempt++;
        } while (!miss && attempt < 100);
        if (attempt == 100) continue;
        T.samples.push_back({i, x, y, -1});
      }
    }
    if (T.samples.empty()) throw std::runtime_error("no training patches");
    std::vector<int> all(T.samples.size());
    for (size_t i = 0; i < all.size(); i++) all[i] = (int)i;
    T.grow(all, 0, 1u);
    *out = h;
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

int oracle_train_hp_tree_size(const oracle_hp_tree* h, int64_t* n_nodes, int64_t* n_leaves, int64_t* i_node,
                              int64_t* n_samples) {
  if (!h) return -1;
  if (n_nodes) *n_nodes = (int64_t)h->t.node_leaf.size();
  if (n_leaves) *n_leaves = (int64_t)h->t.leaf_n.size();
  if (i_node) *i_node = h->t.i_node;
  if (n_samples) *n_samples = (int64_t)h->t.samples.size();
  return 0;
}

int oracle_train_hp_tree_get(const oracle_hp_tree* h, int32_t* node_leaf, int16_t* node_split, double* node_info,
                             int32_t* node_mode, int32_t* leaf_n, float* leaf_fg, int32_t* leaf_labels,
                             int32_t* samples) {
  if (!h) return -1;
  const HPTrainer& t = h->t;
  auto cp = [](auto* dst, const auto& v) {
    if (dst && !v.empty()) std::memcpy(dst, v.data(), v.size() * sizeof(v[0]));
  };
  cp(node_leaf, t.node_leaf);
  cp(node_split, t.node_split);
  cp(node_info, t.node_info);
  cp(node_mode, t.node_mode);
  cp(leaf_n, t.leaf_n);
  cp(leaf_fg, t.leaf_fg);
  cp(leaf_labels, t.leaf_labels);
  if (samples)
    for (size_t i = 0; i < t.samples.size(); i++) {
      samples[4 * i] = t.samples[i].img;
      samples[4 * i + 1] = t.samples[i].x;
      samples[4 * i + 2] = t.samples[i].y;
      samples[4 * i + 3] = t.samples[i].label;
    }
  return 0;
}

void oracle_train_hp_tree_free(oracle_hp_tree* h) { delete h; }

const char* oracle_train_last_error(void) { return g_err.c_str(); }

double oracle_log(double x) { return ffd_log(x); }

}  // extern "C"
