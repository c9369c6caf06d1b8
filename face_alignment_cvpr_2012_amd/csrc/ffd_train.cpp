// ffd_train.cpp — host side of facial-feature tree training (C ABI ffd_train_*, include/ffd.h;
// SURVEY.md §8(f) #3).  Kernels: ffd_train.hip.  CPU restatement (the checker): oracle/ffd_train_oracle.cpp.
//
// The reference grows a Tree<MPSample> depth-first (include/Tree.hpp:102-171), searching each node's
// split over ntests random stripes with a thread pool (SplitGen.hpp:62-101).  Here a whole tree LEVEL is
// one set of launches: every (node, stripe) item of the level is one wave (k_tr_items), the best stripe
// per node is one workgroup (k_tr_select), and the chosen splits re-sort the nodes' sample lists into
// the next level's list (k_tr_partition).  Each node's result depends only on its sample list (in the
// reference's order: the parent's list sorted by the parent's feature value) and its seed, so the
// breadth-first order gives the depth-first tree.  The host keeps the level bookkeeping, builds the
// leaves (MPSample::makeLeaf, MPSample.cpp:146-248: O(samples) per level) and writes the archive.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/ffd.h"
#include "../../include/ffd_gabor.h"
#include "../../include/ffd_model_format.h"
#include "../../include/ffd_numerics.h"
#include "ffd_engine_impl.hpp"
#include "ffd_train.hpp"
#include "model_io.hpp"

namespace ffd_host {
ffd_status archive_model_tree(const ffd::ModelFile& m, int32_t kind, int32_t tree, std::string& out, std::string& err);
}

using namespace ffd_train;

struct ffd_trained_tree {
  int32_t kind = FFD_FOREST_FFD;
  ffd::ModelFile file;  // "mp.*" / "hp.*" arrays of one tree: the archive writer's input
  int64_t n_nodes = 0, n_leaves = 0, n_samples = 0;
  std::vector<int32_t> samples_xy;  // FFD: (image, x, y); head pose: (image, x, y, label)
  std::vector<int32_t> node_mode;   // head pose: split mode per node (-1: leaf)
  ffd_train_stats stats{};
};

namespace {

thread_local std::string g_train_error;

ffd_status fail(ffd_status s, const std::string& m) {
  g_train_error = m;
  return s;
}

constexpr float PATCH_CLOSE_TO_FEATURE = 0.09f;  // Constants.hpp:68
constexpr float LAMDA = 0.125f;                  // MPSample ctor default (MPSample.hpp:38)
constexpr int64_t ITEM_CAP = 1 << 22;            // (node, stripe) items per launch batch

// Boost.Random generate_uniform_int over mt19937 (== boost::mt19937): bucket division with rejection
int uniform_int(std::mt19937& eng, int lo, int hi) {
  const uint32_t range = (uint32_t)(hi - lo);
  if (range == 0) return lo;
  uint32_t bucket = 0xFFFFFFFFu / (range + 1u);
  if (0xFFFFFFFFu % (range + 1u) == range) ++bucket;
  for (;;) {
    const uint32_t r = (uint32_t)eng() / bucket;
    if (r <= range) return lo + (int)r;
  }
}

// SimplePatchFeature::generate (ImageSample.hpp:35-81), host copy of the stripe's draws (the kernels
// draw the same values from k_tr_mt's window)
TrFeature gen_feature(std::mt19937& rng, int ps, int smax) {
  TrFeature f;
  f.ch = uniform_int(rng, 0, ffd_train::NCH - 1);
  f.r[2] = uniform_int(rng, 1, smax);
  f.r[3] = uniform_int(rng, 1, smax);
  f.r[6] = uniform_int(rng, 1, smax);
  f.r[7] = uniform_int(rng, 1, smax);
  f.r[0] = uniform_int(rng, 0, ps - f.r[2] - 1);
  f.r[1] = uniform_int(rng, 0, ps - f.r[3] - 1);
  f.r[4] = uniform_int(rng, 0, ps - f.r[6] - 1);
  f.r[5] = uniform_int(rng, 0, ps - f.r[7] - 1);
  return f;
}

struct HSample {
  int off[10][2];
  float prob[10];
  bool pos;
};

struct NodeRec {
  bool leaf = false;
  int leaf_idx = -1;
  TrFeature f{};
  int thr = 0;
  double info = 0;
};

struct LevelNode {
  uint32_t heap;
  int depth, beg, cnt;
};

struct Leaves {
  std::vector<int32_t> n;
  std::vector<float> fg, var, pf;
  std::vector<int16_t> off;
};

// MPSample::makeLeaf (MPSample.cpp:146-248) over the samples ids[0..n) in list order
int make_leaf(const std::vector<HSample>& S, const int32_t* ids, int n, Leaves& L) {
  const int l = (int)L.n.size();
  L.n.push_back(n);
  for (int j = 0; j < 10; j++) {
    L.off.push_back(0);
    L.off.push_back(0);
    L.var.push_back(FLT_MAX);  // boost::numeric::bounds<float>::highest()
    L.pf.push_back(0.f);
  }
  float fg = 0;
  int size = 0;
  for (int i = 0; i < n; i++) size += S[ids[i]].pos ? 1 : 0;
  if (size > 0) {
    for (int j = 0; j < 10; j++) {
      int mx = 0, my = 0;
      float sum_dist = 0;
      for (int i = 0; i < n; i++) {
        const HSample& s = S[ids[i]];
        if (!s.pos) continue;
        sum_dist += s.prob[j];
        mx += s.off[j][0];
        my += s.off[j][1];
      }
      mx /= size;
      my /= size;
      L.pf[l * 10 + j] = sum_dist / (float)size;
      L.off[(l * 10 + j) * 2] = (int16_t)mx;
      L.off[(l * 10 + j) * 2 + 1] = (int16_t)my;
      double var = 0.0;
      for (int i = 0; i < n; i++) {
        const HSample& s = S[ids[i]];
        if (!s.pos) continue;
        const int x = s.off[j][0], y = s.off[j][1];
        const float dist = (float)std::sqrt((double)((x - mx) * (x - mx) + (y - my) * (y - my)));
        var += dist;
      }
      var /= size;
      L.var[l * 10 + j] = (float)var;
    }
    fg = size / (float)n;
  }
  L.fg.push_back(fg);
  return l;
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Stream {
  hipStream_t s = nullptr;
  ~Stream() { if (s) (void)hipStreamDestroy(s); }
};

// ImageSample(img, {0, 1, 2}, false) of every training image: the 38 exact u32 integral planes into
// d_chan (TrImage::ch_off); gray[i] / stride[i]: image i's rows.  Fills ti[i].gray_off / ch_off.
void build_channels(std::vector<TrImage>& ti, const std::vector<const uint8_t*>& rows, const std::vector<int>& stride,
                    DevBuf& d_chan, hipStream_t s) {
  const int n_img = (int)ti.size();
  int64_t gray_total = 0;
  for (auto& t : ti) { t.gray_off = gray_total; gray_total += (int64_t)t.w * t.h; }
  DevBuf d_gray, d_imgs, d_sep, d_taps, d_u8, d_mag, d_v;
  std::vector<uint8_t> gray((size_t)gray_total);
  for (int i = 0; i < n_img; i++)
    for (int y = 0; y < ti[i].h; y++)
      std::memcpy(&gray[(size_t)ti[i].gray_off + (size_t)y * ti[i].w], rows[i] + (size_t)y * stride[i], ti[i].w);
  upload(d_gray, gray, s);
  int64_t ch_total = 0;
  for (auto& t : ti) { t.ch_off = ch_total; ch_total += (int64_t)ffd_train::NCH * (t.w + 1) * (t.h + 1); }
  d_chan.ensure((size_t)ch_total * 4);
  std::vector<ffd_gabor_sep> sep(5);
  std::memset(sep.data(), 0, sizeof(ffd_gabor_sep) * 5);
  for (int nu = 1; nu <= 4; nu++) ffd_gabor_sep_init(nu, &sep[nu]);
  upload(d_sep, sep, s);
  std::vector<float> taps(7 * 98);
  for (int mu = 0; mu < 7; mu++)
    if (ffd_gabor_taps(0, mu, &taps[mu * 98], &taps[mu * 98 + 49]) != 7) throw std::runtime_error("7x7 Gabor taps");
  upload(d_taps, taps, s);
  // channel scratch in batches of images (u8 38 B, mag 140 B, V 144 B per pixel)
  const int64_t batch_px = 64ll << 20;
  for (int b0 = 0; b0 < n_img;) {
    int b1 = b0;
    int64_t px = 0;
    while (b1 < n_img && (b1 == b0 || px + (int64_t)ti[b1].w * ti[b1].h <= batch_px)) {
      px += (int64_t)ti[b1].w * ti[b1].h;
      b1++;
    }
    std::vector<TrImage> bi(ti.begin() + b0, ti.begin() + b1);
    int64_t o = 0;
    for (auto& t : bi) {
      const int64_t n = (int64_t)t.w * t.h;
      t.u8_off = ffd_train::NCH * o;
      t.mag_off = 35 * o;
      t.v_off = 36 * o;
      o += n;
    }
    d_u8.ensure((size_t)ffd_train::NCH * o);
    d_mag.ensure((size_t)35 * o * 4);
    d_v.ensure((size_t)36 * o * 4);
    upload(d_imgs, bi, s);
    int bmax = 0;
    for (auto& t : bi) bmax = std::max(bmax, t.w * t.h);
    launch_channels(d_imgs.as<TrImage>(), (int)bi.size(), bmax, d_gray.as<uint8_t>(), d_sep.as<ffd_gabor_sep>(),
                    d_taps.as<float>(), d_u8.as<uint8_t>(), d_mag.as<float>(), d_v.as<float>(), d_chan.as<uint32_t>(), s);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(s));  // the scratch is reused by the next batch
    b0 = b1;
  }
}

void put_common(ffd::ModelFile& m, const char* P, const ffd_train_param& p, int64_t i_node, uint64_t NN);

// fixed / n_fixed: the caller's patches as (image, x, y) triples (Tree<MPSample>(samples, ...) of a caller that drew
// them itself, train_ffd.cpp:102-111) instead of npatches draws per image from tree_seed
ffd_status train(const ffd_train_param& P, const ffd_train_image* imgs, int n_img, ffd_trained_tree& out,
                 const int32_t* fixed = nullptr, int64_t n_fixed = 0) {
  const double t0 = now_ms();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(FFD_ERR_DEVICE, "no HIP device");
  if (P.device < 0 || P.device >= ndev) return fail(FFD_ERR_INVALID_ARGUMENT, "device ordinal out of range");
  HIP_CHECK(hipSetDevice(P.device));
  Stream st;
  HIP_CHECK(hipStreamCreateWithFlags(&st.s, hipStreamNonBlocking));
  hipStream_t s = st.s;
  const int ps = (int)std::round((float)P.face_size * P.patch_size_ratio);  // ForestParam::getPatchSize
  const int smax = (int)((ps - 1) * 0.75);                                   // SimplePatchFeature::generate
  if (ps < 2 || ps > 64) return fail(FFD_ERR_INVALID_ARGUMENT, "patch size out of range (2..64)");

  // ---- patches + MPSample data (train_ffd.cpp:102-111, MPSample.cpp:13-41) --------------------------
  std::mt19937 rng(P.tree_seed);
  std::vector<TrImage> ti(n_img);
  std::vector<TrSample> ts;
  std::vector<HSample> hs;
  std::vector<float> prob;
  for (int i = 0; i < n_img; i++) {
    const ffd_train_image& im = imgs[i];
    if (!im.gray || !im.parts || im.width < ps + 4 || im.height < ps + 4 || im.stride < im.width || im.width > 4096 ||
        im.height > 4096)
      return fail(FFD_ERR_INVALID_ARGUMENT, "training image " + std::to_string(i) + ": bad size or NULL data");
    ti[i].w = im.width;
    ti[i].h = im.height;
  }
  const int64_t n_draw = fixed ? n_fixed : (int64_t)n_img * P.npatches;
  for (int64_t k = 0; k < n_draw; k++) {
    {
      TrSample t;
      if (fixed) {
        t.img = fixed[3 * k];
        t.x = fixed[3 * k + 1];
        t.y = fixed[3 * k + 2];
        if (t.img < 0 || t.img >= n_img || t.x < 0 || t.y < 0 || t.x + ps > imgs[t.img].width ||
            t.y + ps > imgs[t.img].height)
          return fail(FFD_ERR_INVALID_ARGUMENT, "patch " + std::to_string(k) + " outside its training image");
      } else {
        t.img = (int)(k / P.npatches);
        t.x = uniform_int(rng, 1, imgs[t.img].width - ps - 2);  // rand_x() first (train_ffd.cpp:108)
        t.y = uniform_int(rng, 1, imgs[t.img].height - ps - 2);
      }
      const ffd_train_image& im = imgs[t.img];
      HSample h;
      const int cx = t.x + ps / 2, cy = t.y + ps / 2;
      h.pos = false;
      for (int q = 0; q < 10; q++) {
        h.off[q][0] = im.parts[2 * q] - cx;
        h.off[q][1] = im.parts[2 * q + 1] - cy;
        const float fx = (float)h.off[q][0] / (float)P.face_size, fy = (float)h.off[q][1] / (float)P.face_size;
        const float d = (float)std::sqrt((double)fx * fx + (double)fy * fy);
        h.prob[q] = ffd_expf(-d / LAMDA);
        if (h.prob[q] > PATCH_CLOSE_TO_FEATURE) h.pos = true;
        prob.push_back(h.prob[q]);
      }
      ts.push_back(t);
      hs.push_back(h);
      out.samples_xy.insert(out.samples_xy.end(), {t.img, t.x, t.y});
    }
  }
  const int N = (int)ts.size();
  if (N == 0) return fail(FFD_ERR_INVALID_ARGUMENT, "no training patches (npatches == 0)");
  out.stats.samples = N;

  // ---- channels of every image (ImageSample(img, {0, 1, 2}, false)) ------------------------------
  DevBuf d_imgs, d_chan;
  {
    std::vector<const uint8_t*> rows(n_img);
    std::vector<int> stride(n_img);
    for (int i = 0; i < n_img; i++) { rows[i] = imgs[i].gray; stride[i] = imgs[i].stride; }
    build_channels(ti, rows, stride, d_chan, s);
  }
  upload(d_imgs, ti, s);
  DevBuf d_samples, d_prob, d_list, d_next, d_nodes, d_raw, d_sorted, d_info, d_thr, d_k, d_best, d_feats, d_err;
  upload(d_samples, ts, s);
  upload(d_prob, prob, s);
  {
    std::vector<int32_t> all(N);
    for (int i = 0; i < N; i++) all[i] = i;
    upload(d_list, all, s);
    d_next.ensure((size_t)N * 4);
  }
  d_err.ensure(4);
  HIP_CHECK(hipMemsetAsync(d_err.p, 0, 4, s));
  HIP_CHECK(hipStreamSynchronize(s));
  out.stats.channels_ms = now_ms() - t0;

  // ---- levels -----------------------------------------------------------------------------------
  std::unordered_map<uint32_t, NodeRec> rec;
  Leaves L;
  int64_t i_node = 0;
  auto leaf_inc = [&](int depth) {  // i_node += powf(2, max_depth - depth) - 1 (Tree.hpp:110)
    i_node = (int64_t)((float)i_node + (std::pow(2.0f, (float)(P.max_depth - depth)) - 1.0f));
  };
  std::vector<LevelNode> level{{1u, 0, 0, N}};
  std::vector<int32_t> h_list(N);
  while (!level.empty()) {
    out.stats.levels++;
    HIP_CHECK(hipMemcpyAsync(h_list.data(), d_list.p, (size_t)N * 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    double tl = now_ms();
    std::vector<LevelNode> cand;
    for (const LevelNode& nd : level) {
      if (nd.cnt < P.min_patches || nd.depth >= P.max_depth) {
        NodeRec r;
        r.leaf = true;
        r.leaf_idx = make_leaf(hs, h_list.data() + nd.beg, nd.cnt, L);
        rec[nd.heap] = r;
        leaf_inc(nd.depth);
      } else {
        cand.push_back(nd);
      }
    }
    out.stats.leaves_ms += now_ms() - tl;
    if (cand.empty()) break;
    // split search, in batches of nodes of at most ITEM_CAP items
    const double ts0 = now_ms();
    std::vector<TrBest> best(cand.size());
    for (size_t c0 = 0; c0 < cand.size();) {
      size_t c1 = c0;
      int64_t items = 0, sorted_total = 0;
      std::vector<TrNode> tn;
      while (c1 < cand.size() && (c1 == c0 || items + P.ntests <= ITEM_CAP)) {
        TrNode t;
        t.beg = cand[c1].beg;
        t.cnt = cand[c1].cnt;
        t.heap = cand[c1].heap;
        t.pad = 0;
        t.sorted_off = sorted_total;
        sorted_total += (int64_t)P.ntests * t.cnt;
        items += P.ntests;
        tn.push_back(t);
        c1++;
      }
      upload(d_nodes, tn, s);
      d_raw.ensure((size_t)items * MT_WIN * 4);
      d_sorted.ensure((size_t)sorted_total * 4);
      d_info.ensure((size_t)items * 8);
      d_thr.ensure((size_t)items * 4);
      d_k.ensure((size_t)items * 4);
      d_best.ensure(tn.size() * sizeof(TrBest));
      launch_mt(d_nodes.as<TrNode>(), (int)items, P.ntests, P.split_seed, d_raw.as<uint32_t>(), s);
      TrItemsArgs a;
      a.nodes = d_nodes.as<TrNode>();
      a.n_items = (int)items;
      a.ntests = P.ntests;
      a.nthr = TR_THR;
      a.ps = ps;
      a.smax = smax;
      a.list = d_list.as<int32_t>();
      a.imgs = d_imgs.as<TrImage>();
      a.samples = d_samples.as<TrSample>();
      a.prob = d_prob.as<float>();
      a.chan = d_chan.as<uint32_t>();
      a.raw = d_raw.as<uint32_t>();
      a.sorted = d_sorted.as<int32_t>();
      a.out_info = d_info.as<double>();
      a.out_thr = d_thr.as<int32_t>();
      a.out_k = d_k.as<int32_t>();
      a.error = d_err.as<int>();
      launch_items(a, s);
      launch_select((int)tn.size(), P.ntests, d_info.as<double>(), d_thr.as<int32_t>(), d_k.as<int32_t>(),
                    d_best.as<TrBest>(), s);
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipMemcpyAsync(best.data() + c0, d_best.p, tn.size() * sizeof(TrBest), hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipStreamSynchronize(s));
      out.stats.items += items;
      c0 = c1;
    }
    int err = 0;
    HIP_CHECK(hipMemcpy(&err, d_err.p, 4, hipMemcpyDeviceToHost));
    if (err) return fail(FFD_ERR_INTERNAL, "a stripe's mt19937 draw window ran out (more than 14 rejections)");
    out.stats.search_ms += now_ms() - ts0;
    // leaves where no stripe found a valid split; the chosen splits (Tree.hpp:135-166)
    const double tp0 = now_ms();
    std::vector<LevelNode> next;
    std::vector<TrNode> pn;
    std::vector<TrFeature> pf;
    for (size_t i = 0; i < cand.size(); i++) {
      const LevelNode& nd = cand[i];
      const TrBest& b = best[i];
      NodeRec r;
      if (b.stripe < 0) {
        r.leaf = true;
        r.leaf_idx = make_leaf(hs, h_list.data() + nd.beg, nd.cnt, L);
        rec[nd.heap] = r;
        leaf_inc(nd.depth);
        continue;
      }
      std::mt19937 srng((uint32_t)((uint64_t)(b.stripe + 1) * (uint64_t)(P.split_seed + nd.heap)));
      r.f = gen_feature(srng, ps, smax);
      r.thr = b.thr;
      r.info = b.info;
      rec[nd.heap] = r;
      i_node++;
      if (b.k < 2 || b.k > nd.cnt - 2) return fail(FFD_ERR_INTERNAL, "split point out of range");
      next.push_back({2 * nd.heap, nd.depth + 1, nd.beg, b.k});
      next.push_back({2 * nd.heap + 1, nd.depth + 1, nd.beg + b.k, nd.cnt - b.k});
      TrNode t{nd.beg, nd.cnt, nd.heap, 0, 0};
      pn.push_back(t);
      pf.push_back(r.f);
    }
    if (!pn.empty()) {
      upload(d_nodes, pn, s);
      upload(d_feats, pf, s);
      launch_partition((int)pn.size(), d_nodes.as<TrNode>(), d_feats.as<TrFeature>(), d_imgs.as<TrImage>(),
                       d_samples.as<TrSample>(), d_chan.as<uint32_t>(), d_list.as<int32_t>(), d_next.as<int32_t>(), s);
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipStreamSynchronize(s));
      std::swap(d_list.p, d_next.p);
      std::swap(d_list.n, d_next.n);
    }
    out.stats.partition_ms += now_ms() - tp0;
    level.swap(next);
  }

  // ---- pre-order arrays (TreeNode::serialize order: node, left subtree, right subtree) ------------
  std::vector<int32_t> node_leaf;
  std::vector<int16_t> node_split;
  std::vector<double> node_info;
  std::vector<uint32_t> stack{1u};
  while (!stack.empty()) {
    const uint32_t h = stack.back();
    stack.pop_back();
    auto it = rec.find(h);
    if (it == rec.end()) return fail(FFD_ERR_INTERNAL, "tree node missing");
    const NodeRec& r = it->second;
    node_leaf.push_back(r.leaf ? r.leaf_idx : -1);
    const int16_t sp[10] = {(int16_t)r.f.ch,   (int16_t)r.f.r[0], (int16_t)r.f.r[1], (int16_t)r.f.r[2], (int16_t)r.f.r[3],
                            (int16_t)r.f.r[4], (int16_t)r.f.r[5], (int16_t)r.f.r[6], (int16_t)r.f.r[7], (int16_t)r.thr};
    if (r.leaf)
      for (int j = 0; j < 10; j++) node_split.push_back(0);
    else
      node_split.insert(node_split.end(), sp, sp + 10);
    node_info.push_back(r.leaf ? 0.0 : r.info);
    if (!r.leaf) {
      stack.push_back(2 * h + 1);
      stack.push_back(2 * h);
    }
  }
  // leaf ordinals in pre-order (the archive writer emits leaves as it meets them)
  {
    std::vector<int32_t> remap(L.n.size(), -1);
    int next_l = 0;
    for (auto& v : node_leaf)
      if (v >= 0) { remap[v] = next_l; v = next_l++; }
    Leaves R;
    R.n.resize(L.n.size());
    R.fg.resize(L.n.size());
    R.var.resize(L.var.size());
    R.pf.resize(L.pf.size());
    R.off.resize(L.off.size());
    for (size_t l = 0; l < L.n.size(); l++) {
      const int d = remap[l];
      R.n[d] = L.n[l];
      R.fg[d] = L.fg[l];
      for (int j = 0; j < 10; j++) {
        R.var[d * 10 + j] = L.var[l * 10 + j];
        R.pf[d * 10 + j] = L.pf[l * 10 + j];
        R.off[(d * 10 + j) * 2] = L.off[(l * 10 + j) * 2];
        R.off[(d * 10 + j) * 2 + 1] = L.off[(l * 10 + j) * 2 + 1];
      }
    }
    L = std::move(R);
  }
  const uint64_t NN = node_leaf.size(), NL = L.n.size();
  ffd::ModelFile& m = out.file;
  m.put<int32_t>("mp.node_leaf", "i32", {NN}, node_leaf);
  m.put<int16_t>("mp.node_split", "i16", {NN, FFD_SPLIT_FIELDS}, node_split);
  m.put<double>("mp.node_info", "f64", {NN}, node_info);
  m.put<int32_t>("mp.leaf_n", "i32", {NL}, L.n);
  m.put<float>("mp.leaf_fg", "f32", {NL}, L.fg);
  m.put<int16_t>("mp.leaf_offset", "i16", {NL, FFD_NUM_PARTS, 2}, L.off);
  m.put<float>("mp.leaf_var", "f32", {NL, FFD_NUM_PARTS}, L.var);
  m.put<float>("mp.leaf_pf", "f32", {NL, FFD_NUM_PARTS}, L.pf);
  put_common(m, "mp", P, i_node, NN);
  out.n_samples = N;
  out.n_nodes = (int64_t)NN;
  out.n_leaves = (int64_t)NL;
  out.stats.total_ms = now_ms() - t0;
  return FFD_OK;
}


// ---- head pose (train_headpose.cpp, HeadPoseSample.cpp) ------------------------------------------------
// intersect (face_utils.cpp:325-346) is empty
bool hp_disjoint(int ax, int ay, int aw, int ah, int bx, int by, int bw, int bh) {
  const int x = ax < bx ? bx : ax, y = ay < by ? by : ay;
  const int w = (ax + aw < bx + bw ? ax + aw : bx + bw) - x, h = (ay + ah < by + bh ? ay + ah : by + bh) - y;
  return w <= 0 || h <= 0;
}

// the Tree / ForestParam fields of a trained tree's archive (Tree<S>::serialize, Tree.hpp:334-343)
void put_common(ffd::ModelFile& m, const char* P, const ffd_train_param& p, int64_t i_node, uint64_t NN) {
  const std::string k = P;
  m.put<int64_t>(k + ".tree_node_off", "i64", {2}, {0, (int64_t)NN});
  const int64_t m_num_nodes = (int64_t)(std::pow(2.0f, (float)p.max_depth) - 1);  // Tree.hpp:53
  m.put<int64_t>(k + ".tree_counts", "i64", {1, 2}, {m_num_nodes, i_node});
  m.put<int32_t>(k + ".tree_param", "i32", {1, 7},
                 {p.max_depth, p.min_patches, p.ntests, p.ntrees, p.nimages, p.npatches, p.face_size});
  m.put<float>(k + ".tree_ratio", "f32", {1}, {p.patch_size_ratio});
  m.put<int32_t>(k + ".tree_features", "i32", {3}, {0, 1, 2});
  m.put<int64_t>(k + ".tree_features_off", "i64", {2}, {0, 3});
  std::vector<uint8_t> str;
  std::vector<int64_t> str_off{0};
  for (const char* t : {p.tree_path, p.image_path, p.save_path}) {
    const std::string v = t ? t : "";
    str.insert(str.end(), v.begin(), v.end());
    str_off.push_back((int64_t)str.size());
  }
  m.put<uint8_t>(k + ".tree_strings", "u8", {(uint64_t)str.size()}, str);
  m.put<int64_t>(k + ".tree_strings_off", "i64", {4}, str_off);
}

// Tree<HeadPoseSample> growth.  The split mode of a searched node is the tree generator's next draw in
// depth-first order (Tree.hpp:267-274), so the nodes are searched one at a time in that order: every
// stripe of the node at once (k_hp_items, one workgroup per stripe), then the node's best split and its
// two sample lists (k_hp_split), one host round trip per searched node.  A node at depth d keeps its list
// in lists[d]; its children go to lists[d + 1], which holds nothing still pending (the depth-first
// stack's pending nodes are right siblings on the current path, at depth <= d).
ffd_status train_hp(const ffd_train_param& P, const ffd_train_hp_image* imgs, int n_img, ffd_trained_tree& out) {
  const double t0 = now_ms();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(FFD_ERR_DEVICE, "no HIP device");
  if (P.device < 0 || P.device >= ndev) return fail(FFD_ERR_INVALID_ARGUMENT, "device ordinal out of range");
  HIP_CHECK(hipSetDevice(P.device));
  Stream st;
  HIP_CHECK(hipStreamCreateWithFlags(&st.s, hipStreamNonBlocking));
  hipStream_t s = st.s;
  const int ps = (int)std::round((float)P.face_size * P.patch_size_ratio);  // ForestParam::getPatchSize
  const int smax = (int)((ps - 1) * 0.75);
  if (ps < 2 || ps > 64 || P.face_size <= ps) return fail(FFD_ERR_INVALID_ARGUMENT, "patch / face size out of range");

  // ---- patches (train_headpose.cpp:98-134); draws from the tree generator, x before y ------------------
  std::mt19937 rng(P.tree_seed);
  std::vector<TrImage> ti(n_img);
  std::vector<TrSample> ts;
  std::vector<int8_t> cls;
  for (int i = 0; i < n_img; i++) {
    const ffd_train_hp_image& im = imgs[i];
    const ffd_rect& b = im.face;
    if (!im.gray || im.width < ps + 1 || im.height < ps + 1 || im.stride < im.width || im.width > 4096 ||
        im.height > 4096 || b.x < 0 || b.y < 0 || b.x + P.face_size - 1 > im.width ||
        b.y + P.face_size - 1 > im.height || im.pose < -2 || im.pose > 2)
      return fail(FFD_ERR_INVALID_ARGUMENT, "training image " + std::to_string(i) + ": bad size, face box or pose");
    ti[i].w = im.width;
    ti[i].h = im.height;
    for (int j = 0; j < P.npatches * (1 - 0.2f); j++) {  // NEG_PATCHES_RATIO 0.2f
      TrSample t;
      t.img = i;
      t.x = b.x + uniform_int(rng, 0, P.face_size - ps - 1);
      t.y = b.y + uniform_int(rng, 0, P.face_size - ps - 1);
      ts.push_back(t);
      cls.push_back((int8_t)(im.pose + 2));
      out.samples_xy.insert(out.samples_xy.end(), {t.img, t.x, t.y, im.pose + 2});
    }
    for (int j = 0; j < P.npatches * 0.2f; j++) {
      int x, y, attempt = 0;
      bool miss;
      do {  // MAX_NEG_ATTEMPTS 100
        x = uniform_int(rng, 0, im.width - ps - 1);
        y = uniform_int(rng, 0, im.height - ps - 1);
        miss = hp_disjoint(x, y, ps, ps, b.x, b.y, b.width, b.height);
        attempt++;
      } while (!miss && attempt < 100);
      if (attempt == 100) continue;
      ts.push_back({i, x, y});
      cls.push_back(5);
      out.samples_xy.insert(out.samples_xy.end(), {i, x, y, -1});
    }
  }
  const int N = (int)ts.size();
  if (N == 0) return fail(FFD_ERR_INVALID_ARGUMENT, "no training patches (npatches == 0)");
  out.stats.samples = N;
  out.n_samples = N;

  DevBuf d_imgs, d_chan;
  {
    std::vector<const uint8_t*> rows(n_img);
    std::vector<int> stride(n_img);
    for (int i = 0; i < n_img; i++) { rows[i] = imgs[i].gray; stride[i] = imgs[i].stride; }
    build_channels(ti, rows, stride, d_chan, s);
  }
  upload(d_imgs, ti, s);
  DevBuf d_samples, d_cls, d_lists, d_info, d_thr, d_res, d_err;
  upload(d_samples, ts, s);
  upload(d_cls, cls, s);
  d_lists.ensure((size_t)(P.max_depth + 1) * N * 4);
  std::vector<int32_t> all(N);
  for (int i = 0; i < N; i++) all[i] = i;
  HIP_CHECK(hipMemcpyAsync(d_lists.p, all.data(), (size_t)N * 4, hipMemcpyHostToDevice, s));
  d_info.ensure((size_t)P.ntests * 8);
  d_thr.ensure((size_t)P.ntests * 4);
  d_res.ensure(sizeof(HpSplitResult));
  d_err.ensure(4);
  HIP_CHECK(hipMemsetAsync(d_err.p, 0, 4, s));
  HpSplitResult* h_res = nullptr;
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_res), sizeof(HpSplitResult), hipHostMallocDefault));
  struct Pinned {
    void* p;
    ~Pinned() { if (p) (void)hipHostFree(p); }
  } pinned{h_res};
  HIP_CHECK(hipStreamSynchronize(s));
  out.stats.channels_ms = now_ms() - t0;

  // ---- depth-first growth (Tree.hpp:102-171) ------------------------------------------------------
  struct Frame {
    uint32_t heap;
    int depth, off, n;
    int hist[6];  // labels 0..4, background
  };
  std::vector<int32_t> node_leaf, node_mode, leaf_n, leaf_labels;
  std::vector<int16_t> node_split;
  std::vector<double> node_info;
  std::vector<float> leaf_fg;
  int64_t i_node = 0;
  auto make_leaf = [&](const Frame& f) {  // HeadPoseSample::makeLeaf (HeadPoseSample.cpp:89-118)
    int size = 0;
    for (int c = 0; c < 5; c++) size += f.hist[c];
    node_leaf.push_back((int32_t)leaf_n.size());
    leaf_n.push_back(f.n);
    leaf_fg.push_back((float)size / (float)f.n);
    for (int c = 0; c < 5; c++) leaf_labels.push_back(size > 0 ? f.hist[c] : 0);
    for (int j = 0; j < 10; j++) node_split.push_back(0);
    node_info.push_back(0.0);
    node_mode.push_back(-1);
    // i_node += powf(2, max_depth - depth) - 1 (Tree.hpp:110)
    i_node = (int64_t)((float)i_node + (std::pow(2.0f, (float)(P.max_depth - f.depth)) - 1.0f));
  };
  Frame root{1u, 0, 0, N, {0, 0, 0, 0, 0, 0}};
  for (int8_t c : cls) root.hist[(int)c]++;
  std::vector<Frame> stack{root};
  int max_level = 0;
  while (!stack.empty()) {
    const Frame f = stack.back();
    stack.pop_back();
    max_level = std::max(max_level, f.depth + 1);
    if (f.n < P.min_patches || f.depth >= P.max_depth) {
      const double tl = now_ms();
      make_leaf(f);
      out.stats.leaves_ms += now_ms() - tl;
      continue;
    }
    const int mode = uniform_int(rng, 0, 100);  // rand_split() of findOptimalSplit (Tree.hpp:267-274)
    const double ts0 = now_ms();
    const uint32_t T = P.split_seed + f.heap;
    const int32_t* list = d_lists.as<int32_t>() + (size_t)f.depth * N + f.off;
    HpItemsArgs a;
    a.list = list;
    a.n = f.n;
    a.T = T;
    a.mode = mode;
    a.nthr = TR_THR;
    a.ps = ps;
    a.smax = smax;
    a.imgs = d_imgs.as<TrImage>();
    a.samples = d_samples.as<TrSample>();
    a.cls = d_cls.as<int8_t>();
    a.chan = d_chan.as<uint32_t>();
    a.out_info = d_info.as<double>();
    a.out_thr = d_thr.as<int32_t>();
    a.error = d_err.as<int>();
    launch_hp_items(a, P.ntests, s);
    HpSplitArgs b;
    b.ntests = P.ntests;
    b.info = d_info.as<double>();
    b.thr = d_thr.as<int32_t>();
    b.T = T;
    b.ps = ps;
    b.smax = smax;
    b.list = list;
    b.n = f.n;
    b.out = d_lists.as<int32_t>() + (size_t)(f.depth + 1) * N;  // depth < max_depth here
    b.imgs = a.imgs;
    b.samples = a.samples;
    b.cls = a.cls;
    b.chan = a.chan;
    b.res = d_res.as<HpSplitResult>();
    launch_hp_split(b, s);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(h_res, d_res.p, sizeof(HpSplitResult), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    out.stats.items += P.ntests;
    out.stats.search_ms += now_ms() - ts0;
    const HpSplitResult r = *h_res;
    if (r.stripe < 0) {  // no valid split: leaf (Tree.hpp:156-165)
      make_leaf(f);
      continue;
    }
    if (r.bad) return fail(FFD_ERR_INTERNAL, "a stripe's mt19937 draw window ran out (more than 14 rejections)");
    if (r.na < 2 || r.nb < 2 || r.na + r.nb != f.n) return fail(FFD_ERR_INTERNAL, "split sizes out of range");
    node_leaf.push_back(-1);
    const int16_t sp[10] = {(int16_t)r.ch,      (int16_t)r.rect[0], (int16_t)r.rect[1], (int16_t)r.rect[2],
                            (int16_t)r.rect[3], (int16_t)r.rect[4], (int16_t)r.rect[5], (int16_t)r.rect[6],
                            (int16_t)r.rect[7], (int16_t)r.thr};
    node_split.insert(node_split.end(), sp, sp + 10);
    node_info.push_back(r.info);
    node_mode.push_back(mode);
    i_node++;
    Frame L{2 * f.heap, f.depth + 1, 0, r.na, {}}, R{2 * f.heap + 1, f.depth + 1, r.na, r.nb, {}};
    for (int c = 0; c < 6; c++) { L.hist[c] = r.ha[c]; R.hist[c] = r.hb[c]; }
    stack.push_back(R);
    stack.push_back(L);
  }
  int err = 0;
  HIP_CHECK(hipMemcpy(&err, d_err.p, 4, hipMemcpyDeviceToHost));
  if (err) return fail(FFD_ERR_INTERNAL, "a stripe's mt19937 draw window ran out (more than 14 rejections)");
  out.stats.levels = max_level;
  const uint64_t NN = node_leaf.size(), NL = leaf_n.size();
  ffd::ModelFile& m = out.file;
  m.put<int32_t>("hp.node_leaf", "i32", {NN}, node_leaf);
  m.put<int16_t>("hp.node_split", "i16", {NN, FFD_SPLIT_FIELDS}, node_split);
  m.put<double>("hp.node_info", "f64", {NN}, node_info);
  m.put<int32_t>("hp.leaf_n", "i32", {NL}, leaf_n);
  m.put<float>("hp.leaf_fg", "f32", {NL}, leaf_fg);
  m.put<int32_t>("hp.leaf_labels", "i32", {NL, FFD_NUM_HP_LABELS}, leaf_labels);
  put_common(m, "hp", P, i_node, NN);
  out.kind = FFD_FOREST_HEADPOSE;
  out.node_mode = std::move(node_mode);
  out.n_nodes = (int64_t)NN;
  out.n_leaves = (int64_t)NL;
  out.stats.total_ms = now_ms() - t0;
  return FFD_OK;
}

}  // namespace

extern "C" {

void ffd_train_param_init(ffd_train_param* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->max_depth = 20;
  p->min_patches = 20;
  p->ntests = 2500;
  p->ntrees = 20;
  p->nimages = 600;
  p->npatches = 150;
  p->face_size = 125;
  p->patch_size_ratio = 0.25f;
  p->tree_path = "data/trees_ffd";
  p->image_path = "../../database/faces/lfw/lfw_ffd_ann.txt";
  p->save_path = "data/trees_ffd/forest_0/tree_000.txt";
  p->tree_seed = 1;
  p->split_seed = 1;
  p->device = 0;
}

ffd_status ffd_train_mp_tree(const ffd_train_param* p, const ffd_train_image* images, int32_t n_images,
                             ffd_trained_tree** out) {
  return ffd_train_mp_tree_patches(p, images, n_images, nullptr, 0, out);
}

ffd_status ffd_train_mp_tree_patches(const ffd_train_param* p, const ffd_train_image* images, int32_t n_images,
                                     const int32_t* patches, int64_t n_patches, ffd_trained_tree** out) {
  if (!p || !images || !out || n_images <= 0 || n_patches < 0 || (n_patches && !patches))
    return fail(FFD_ERR_INVALID_ARGUMENT, "bad arguments");
  *out = nullptr;
  if (p->max_depth < 1 || p->max_depth > 24 || p->min_patches < 1 || p->ntests < 1 || p->npatches < 0 ||
      p->face_size < 1 || !(p->patch_size_ratio > 0))
    return fail(FFD_ERR_INVALID_ARGUMENT, "ForestParam out of range");
  auto* t = new (std::nothrow) ffd_trained_tree;
  if (!t) return fail(FFD_ERR_OUT_OF_MEMORY, "out of host memory");
  ffd_status st;
  try {
    st = train(*p, images, n_images, *t, patches, n_patches);
  } catch (const HipError& e) {
    st = fail(FFD_ERR_DEVICE, e.what());
  } catch (const std::bad_alloc&) {
    st = fail(FFD_ERR_OUT_OF_MEMORY, "out of host memory");
  } catch (const std::exception& e) {
    st = fail(FFD_ERR_INTERNAL, e.what());
  }
  if (st != FFD_OK) {
    delete t;
    return st;
  }
  *out = t;
  return FFD_OK;
}

void ffd_train_hp_param_init(ffd_train_param* p) {  // data/config_headpose.txt
  ffd_train_param_init(p);
  if (!p) return;
  p->max_depth = 15;
  p->min_patches = 20;
  p->ntests = 2000;
  p->ntrees = 15;
  p->nimages = 400;
  p->npatches = 200;
  p->tree_path = "data/trees_headpose";
  p->save_path = "data/trees_headpose/tree_000.txt";
}

ffd_status ffd_train_hp_tree(const ffd_train_param* p, const ffd_train_hp_image* images, int32_t n_images,
                             ffd_trained_tree** out) {
  if (!p || !images || !out || n_images <= 0) return fail(FFD_ERR_INVALID_ARGUMENT, "bad arguments");
  *out = nullptr;
  if (p->max_depth < 1 || p->max_depth > 24 || p->min_patches < 1 || p->ntests < 1 || p->npatches < 0 ||
      p->face_size < 1 || !(p->patch_size_ratio > 0))
    return fail(FFD_ERR_INVALID_ARGUMENT, "ForestParam out of range");
  auto* t = new (std::nothrow) ffd_trained_tree;
  if (!t) return fail(FFD_ERR_OUT_OF_MEMORY, "out of host memory");
  ffd_status st;
  try {
    st = train_hp(*p, images, n_images, *t);
  } catch (const HipError& e) {
    st = fail(FFD_ERR_DEVICE, e.what());
  } catch (const std::bad_alloc&) {
    st = fail(FFD_ERR_OUT_OF_MEMORY, "out of host memory");
  } catch (const std::exception& e) {
    st = fail(FFD_ERR_INTERNAL, e.what());
  }
  if (st != FFD_OK) {
    delete t;
    return st;
  }
  *out = t;
  return FFD_OK;
}

int32_t ffd_trained_tree_kind(const ffd_trained_tree* t) { return t ? t->kind : -1; }
int64_t ffd_trained_tree_num_samples(const ffd_trained_tree* t) { return t ? t->n_samples : -1; }

ffd_status ffd_trained_tree_hp_arrays(const ffd_trained_tree* t, int32_t* node_leaf, int16_t* node_split,
                                      double* node_info, int32_t* node_mode, int32_t* leaf_n, float* leaf_fg,
                                      int32_t* leaf_labels, int32_t* samples) {
  if (!t) return fail(FFD_ERR_INVALID_ARGUMENT, "tree is NULL");
  if (t->kind != FFD_FOREST_HEADPOSE) return fail(FFD_ERR_INVALID_ARGUMENT, "not a head-pose tree");
  auto cp = [&](void* dst, const char* name) {
    if (!dst) return;
    const auto& a = t->file.get(name);
    if (!a.bytes.empty()) std::memcpy(dst, a.bytes.data(), a.bytes.size());
  };
  cp(node_leaf, "hp.node_leaf");
  cp(node_split, "hp.node_split");
  cp(node_info, "hp.node_info");
  cp(leaf_n, "hp.leaf_n");
  cp(leaf_fg, "hp.leaf_fg");
  cp(leaf_labels, "hp.leaf_labels");
  if (node_mode && !t->node_mode.empty()) std::memcpy(node_mode, t->node_mode.data(), t->node_mode.size() * 4);
  if (samples && !t->samples_xy.empty()) std::memcpy(samples, t->samples_xy.data(), t->samples_xy.size() * 4);
  return FFD_OK;
}

const char* ffd_train_last_error(void) { return g_train_error.c_str(); }

int64_t ffd_trained_tree_num_nodes(const ffd_trained_tree* t) { return t ? t->n_nodes : -1; }
int64_t ffd_trained_tree_num_leaves(const ffd_trained_tree* t) { return t ? t->n_leaves : -1; }

ffd_status ffd_trained_tree_arrays(const ffd_trained_tree* t, int32_t* node_leaf, int16_t* node_split,
                                   double* node_info, int32_t* leaf_n, float* leaf_fg, int16_t* leaf_offset,
                                   float* leaf_var, float* leaf_pf, int32_t* samples_xy) {
  if (!t) return fail(FFD_ERR_INVALID_ARGUMENT, "tree is NULL");
  if (t->kind != FFD_FOREST_FFD) return fail(FFD_ERR_INVALID_ARGUMENT, "not a facial-feature tree");
  auto cp = [&](void* dst, const char* name) {
    if (!dst) return;
    const auto& a = t->file.get(name);
    if (!a.bytes.empty()) std::memcpy(dst, a.bytes.data(), a.bytes.size());
  };
  cp(node_leaf, "mp.node_leaf");
  cp(node_split, "mp.node_split");
  cp(node_info, "mp.node_info");
  cp(leaf_n, "mp.leaf_n");
  cp(leaf_fg, "mp.leaf_fg");
  cp(leaf_offset, "mp.leaf_offset");
  cp(leaf_var, "mp.leaf_var");
  cp(leaf_pf, "mp.leaf_pf");
  if (samples_xy && !t->samples_xy.empty())
    std::memcpy(samples_xy, t->samples_xy.data(), t->samples_xy.size() * 4);
  return FFD_OK;
}

ffd_status ffd_trained_tree_stats(const ffd_trained_tree* t, ffd_train_stats* stats) {
  if (!t || !stats) return fail(FFD_ERR_INVALID_ARGUMENT, "bad arguments");
  *stats = t->stats;
  return FFD_OK;
}

ffd_status ffd_trained_tree_archive(const ffd_trained_tree* t, char* buf, int64_t cap, int64_t* size) {
  if (!t || !size) return fail(FFD_ERR_INVALID_ARGUMENT, "bad arguments");
  std::string s, err;
  const ffd_status st = ffd_host::archive_model_tree(t->file, t->kind, 0, s, err);
  if (st != FFD_OK) return fail(st, err);
  *size = (int64_t)s.size();
  if (!buf) return FFD_OK;
  if (cap < (int64_t)s.size()) return fail(FFD_ERR_INVALID_ARGUMENT, "buffer too small");
  std::memcpy(buf, s.data(), s.size());
  return FFD_OK;
}

ffd_status ffd_trained_tree_save(const ffd_trained_tree* t, const char* path) {
  if (!t || !path) return fail(FFD_ERR_INVALID_ARGUMENT, "bad arguments");
  std::string s, err;
  const ffd_status st = ffd_host::archive_model_tree(t->file, t->kind, 0, s, err);
  if (st != FFD_OK) return fail(st, err);
  FILE* f = std::fopen(path, "wb");
  if (!f) return fail(FFD_ERR_INVALID_ARGUMENT, std::string("cannot write ") + path);
  const bool ok = std::fwrite(s.data(), 1, s.size(), f) == s.size();
  if (std::fclose(f) != 0 || !ok) return fail(FFD_ERR_INTERNAL, std::string("write failed: ") + path);
  return FFD_OK;
}

void ffd_trained_tree_free(ffd_trained_tree* t) { delete t; }

}  // extern "C"
