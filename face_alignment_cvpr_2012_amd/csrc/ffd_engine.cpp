// ffd_engine.cpp — host side of the MI355X engine behind include/ffd.h.
//
// Owns the device-resident model (flattened forests + leaf tables), the workspace
// and one HIP stream; orchestrates the kernel pipeline of ffd_kernels.hip for a batch
// of faces.  Replaces, per reference file (paths relative to /root/reference):
//   FaceForest::FaceForest / Forest::load      src/FaceForest.cpp:15-58, include/Forest.hpp:103-153
//   FaceForest::analyzeFace (batched)          src/FaceForest.cpp:183-258
//   FeatureChannelFactory::initGaborKernels    include/FeatureChannelFactory.hpp:186-251
// The product never calls the CPU oracle; when no HIP device is usable every entry
// point fails with FFD_ERR_DEVICE (no CPU fallback).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ffd.h"
#include "ffd_device.hpp"
#include "ffd_kernels.hpp"
#include "../../include/ffd_gabor.h"
#include "model_io.hpp"
#include "ffd_engine_impl.hpp"

#define FFD_VERSION_STR "ffd-mi355x 0.1.0 (gfx950)"

namespace {

using namespace ffd;
using namespace ffd_host;

// Device integrals are kept modulo 2^16; the u8 plane is the exact mod-2^16 second difference,
// from which the full 32-bit integral ([NCH][H+1][W+1], the reference's layout) is rebuilt.
void widen_integrals(const uint16_t* J, int64_t plane, int W, int H, uint32_t* out) {
  const size_t ow = (size_t)W + 1, oplane = ((size_t)H + 1) * ow;
  for (int c = 0; c < NCH; c++) {
    const uint16_t* j = J + c * plane;
    uint32_t* o = out + c * oplane;
    for (int x = 0; x <= W; x++) o[x] = 0;
    for (int y = 0; y < H; y++) {
      uint32_t run = 0;
      o[(y + 1) * ow] = 0;
      for (int x = 0; x < W; x++) {
        // (signed: a float-integral face's rounded values have second differences in [-16, 271])
        const int16_t v = (int16_t)(uint16_t)(j[(y + 1) * PITCH + x + 1] - j[y * PITCH + x + 1] - j[(y + 1) * PITCH + x] +
                                              j[y * PITCH + x]);
        run += (uint32_t)(int32_t)v;
        o[(y + 1) * ow + x + 1] = o[y * ow + x + 1] + run;
      }
    }
  }
}

// Traversal workgroups per face: one per gx x gy block of the face's patch grid (max over the chunk).
int blocks_per_face(const std::vector<FaceDesc>& fds, bool hp, TravShape g) {
  int m = 0;
  for (const auto& f : fds)
    if (f.valid && !f.fint) {  // float-integral faces are walked by k_walk_fint
      const int nx = hp ? f.nhx : f.nmx, ny = hp ? f.nhy : f.nmy;
      m = std::max(m, ((nx + g.gx - 1) / g.gx) * ((ny + g.gy - 1) / g.gy));
    }
  return m;
}

}  // namespace

namespace {

thread_local std::string g_create_err;

// Flatten the pre-order archive records of every tree into breadth-first node arrays
// with adjacent children (see ffd_device.hpp for the 16-byte node encoding).
void flatten_forest(const ModelFile& m, const std::string& p, std::vector<uint4>& nodes, std::vector<int32_t>& roots,
                    std::vector<int32_t>& sizes) {
  const auto& off = m.get(p + ".tree_node_off");
  const auto& nl = m.get(p + ".node_leaf");
  const auto& ns = m.get(p + ".node_split");
  const int64_t* to = off.as<int64_t>();
  const int32_t* leaf = nl.as<int32_t>();
  const int16_t* sp = ns.as<int16_t>();
  const int64_t T = (int64_t)off.count() - 1;
  nodes.clear();
  roots.clear();
  sizes.clear();
  nodes.reserve(nl.count());
  for (int64_t t = 0; t < T; t++) {
    const int64_t b = to[t], e = to[t + 1];
    const int64_t n = e - b;
    std::vector<int64_t> left(n, -1), right(n, -1), stack;
    for (int64_t i = 0; i < n; i++) {
      if (i > 0) {
        if (stack.empty()) throw std::runtime_error("malformed tree in model");
        int64_t par = stack.back();
        if (left[par] < 0) left[par] = i;
        else { right[par] = i; stack.pop_back(); }
      }
      if (leaf[b + i] < 0) stack.push_back(i);
    }
    if (!stack.empty()) throw std::runtime_error("incomplete tree in model");
    std::vector<int64_t> order{0}, newidx(n, -1);
    for (size_t k = 0; k < order.size(); k++) {
      int64_t v = order[k];
      if (leaf[b + v] < 0) { order.push_back(left[v]); order.push_back(right[v]); }
    }
    const int64_t base = (int64_t)nodes.size();
    for (size_t k = 0; k < order.size(); k++) newidx[order[k]] = base + (int64_t)k;
    roots.push_back((int32_t)base);
    sizes.push_back((int32_t)order.size());
    for (size_t k = 0; k < order.size(); k++) {
      const int64_t v = order[k];
      uint4 nd;
      if (leaf[b + v] >= 0) {
        nd.x = LEAF_BIT | (uint32_t)leaf[b + v];
        nd.y = nd.z = nd.w = 0;
      } else {
        const int16_t* s = sp + (b + v) * FFD_SPLIT_FIELDS;
        const int ch = s[0], x1 = s[1], y1 = s[2], w1 = s[3], h1 = s[4], x2 = s[5], y2 = s[6], w2 = s[7], h2 = s[8];
        if (ch < 0 || ch >= NCH) throw std::runtime_error("split channel out of range");
        // sides <= 22 (SimplePatchFeature::generate, ImageSample.hpp:42-72): the u16 integrals sum a
        // rectangle as two halves of <= 22 x 11 pixels (exact mod 2^16) and the evalTest quotient
        // fma(R, rcp(area), 0.00075) is proven exact for areas <= 484 (tests/test_numerics.py)
        for (int q : {w1, h1, w2, h2})
          if (q < 1 || q > 22) throw std::runtime_error("split rectangle side outside [1, 22] (unsupported model)");
        for (int q : {x1, y1, x2, y2})
          if (q < 0 || q > 31) throw std::runtime_error("split rectangle offset out of range");
        if (x1 + w1 > 31 || y1 + h1 > 31 || x2 + w2 > 31 || y2 + h2 > 31)
          throw std::runtime_error("split rectangle leaves the patch");
        nd.x = (uint32_t)newidx[left[v]];
        if (newidx[right[v]] != newidx[left[v]] + 1) throw std::runtime_error("BFS layout error");
        nd.y = (uint32_t)ch | (uint32_t)w1 << 6 | (uint32_t)h1 << 11 | (uint32_t)w2 << 16 | (uint32_t)h2 << 21;
        nd.z = (uint32_t)(int32_t)s[9];
        nd.w = (uint32_t)(y1 * PITCH + x1) | (uint32_t)(y2 * PITCH + x2) << 16;
      }
      nodes.push_back(nd);
    }
  }
  if ((int64_t)nodes.size() != (int64_t)nl.count()) throw std::runtime_error("node count mismatch");
}

}  // namespace

// One node's 56-bit test (ffd_device.hpp "pair records"): lo 32 bits, hi 24 bits.
static void encode_test(const uint4& n, uint32_t& lo, uint32_t& hi) {
  if (n.x & LEAF_BIT) {
    const uint64_t ord = n.x & ~LEAF_BIT;
    lo = (uint32_t)(ord & 0xFFFFFu) | 63u << 26;
    hi = (uint32_t)(ord >> 20) & 0xFFFFFFu;
    return;
  }
  const uint32_t ch = n.y & 63u, w1 = (n.y >> 6) & 31u, h1 = (n.y >> 11) & 31u, w2 = (n.y >> 16) & 31u,
                 h2 = (n.y >> 21) & 31u;
  const uint32_t e1 = n.w & 0xFFFFu, e2 = n.w >> 16;
  const uint32_t x1 = e1 % PITCH, y1 = e1 / PITCH, x2 = e2 % PITCH, y2 = e2 / PITCH;
  const int thr = (int)n.z;
  if (ch >= 63 || x1 > 31 || y1 > 31 || x2 > 31 || y2 > 31 || w1 < 1 || w1 > 22 || h1 < 1 || h1 > 22 || w2 < 1 ||
      w2 > 22 || h2 < 1 || h2 > 22 || thr < -512 || thr > 511)
    throw std::runtime_error("split outside the pair-record encoding");
  const uint32_t t = (uint32_t)thr & 0x3FFu;
  lo = x1 | y1 << 5 | x2 << 10 | y2 << 15 | (t & 63u) << 20 | ch << 26;  // ch on top: leaf = lo >= 63 << 26
  hi = w1 | h1 << 5 | w2 << 10 | h2 << 15 | (t >> 6) << 20;  // sides as they are: no +1 in the walk
}

// Depth-first pair layout: a pair (a, b) is followed by the pair of a's children and a's whole
// subtree, then b's children pair at offset off1 (16 bits; 0 = look up far[pair]).  Each tree starts
// with a root pair (root, unused leaf).  Leaves keep their model ordinals; speed-neutral for parity:
// every walk visits the same nodes in the same order as Tree<S>::evaluateMT.
void ffd_host::build_pair_records(const std::vector<uint4>& bfs, const std::vector<int32_t>& roots,
                                  std::vector<uint4>& out, std::vector<int32_t>& roots_out,
                                  std::vector<uint32_t>& far) {
  out.clear();
  roots_out.clear();
  far.clear();
  const uint4 unused_leaf = make_uint4(LEAF_BIT, 0u, 0u, 0u);
  auto pack = [](const uint4& a, const uint4& b, uint32_t o16) {
    uint32_t lo0, hi0, lo1, hi1;
    encode_test(a, lo0, hi0);
    encode_test(b, lo1, hi1);
    return make_uint4(lo0, lo1, hi0 | (o16 & 0xFFu) << 24, hi1 | (o16 >> 8) << 24);
  };
  // iterative DFS: a frame places pair (a, b); phase 0 = a's children, 1 = b's children, 2 = done
  struct Frame { uint4 a, b; size_t idx; int phase; };
  for (int32_t root : roots) {
    std::vector<Frame> st;
    roots_out.push_back((int32_t)out.size());
    st.push_back({bfs[(uint32_t)root], unused_leaf, out.size(), 0});
    out.push_back(make_uint4(0, 0, 0, 0));
    far.push_back(0);
    while (!st.empty()) {
      Frame& f = st.back();
      if (f.phase == 0) {
        f.phase = 1;
        if (!(f.a.x & LEAF_BIT)) {
          const uint32_t c = f.a.x;
          st.push_back({bfs[c], bfs[c + 1], out.size(), 0});
          out.push_back(make_uint4(0, 0, 0, 0));
          far.push_back(0);
        }
        continue;
      }
      if (f.phase == 1) {
        f.phase = 2;
        const uint64_t off1 = out.size() - f.idx;  // where b's children pair goes
        uint32_t o16 = off1 <= 0xFFFFu ? (uint32_t)off1 : 0u;
        if (o16 == 0 && !(f.b.x & LEAF_BIT)) far[f.idx] = (uint32_t)off1;
        if (off1 > 0xFFFFFFFFull) throw std::runtime_error("pair array too large");
        out[f.idx] = pack(f.a, f.b, o16);
        if (!(f.b.x & LEAF_BIT)) {
          const uint32_t c = f.b.x;
          const size_t at = out.size();
          out.push_back(make_uint4(0, 0, 0, 0));
          far.push_back(0);
          st.push_back({bfs[c], bfs[c + 1], at, 0});
        }
        continue;
      }
      st.pop_back();
    }
  }
  if (out.size() >= 0x80000000ull) throw std::runtime_error("pair array too large");
}

void ffd_host::build_tree_tops(const std::vector<uint4>& pairs, const std::vector<int32_t>& proots,
                               const std::vector<uint32_t>& far, std::vector<uint4>& tops,
                               std::vector<uint32_t>& top_idx) {
  tops.assign(proots.size() * TOP_CAP, make_uint4(0, 0, 0, 0));
  top_idx.assign(proots.size() * TOP_CAP, 0u);
  auto leaf = [](uint32_t lo) { return (lo >> 26) == 63u; };
  for (size_t t = 0; t < proots.size(); t++) {
    uint4* rec = &tops[t * TOP_CAP];
    uint32_t* idx = &top_idx[t * TOP_CAP];  // pair index of each entry
    idx[0] = (uint32_t)proots[t];
    rec[0] = pairs[idx[0]];
    std::vector<bool> live(TOP_CAP, false);
    live[0] = true;
    for (int h = 0; h < TOP_CAP; h++) {
      if (!live[h]) continue;
      const uint4 R = rec[h];
      const uint32_t p = idx[h];
      for (uint32_t s = 0; s < (h ? 2u : 1u); s++) {  // the root pair's second slot is an unused leaf
        if (leaf(s ? R.y : R.x)) continue;
        const int h2 = h ? 2 * h + (int)s : 1;
        if (h2 >= TOP_CAP) continue;
        const uint32_t off1 = (R.z >> 24) | ((R.w >> 24) << 8);
        const uint32_t q = p + (s ? (off1 ? off1 : far[p]) : 1u);
        rec[h2] = pairs[q];
        idx[h2] = q;
        live[h2] = true;
      }
    }
  }
}

void ffd_engine::load_model(const std::string& path) {
  ModelFile m;
  m.load(path);
  const int32_t* hp_param = m.get("hp.param").as<int32_t>();
  const int32_t* mp_param = m.get("mp.param").as<int32_t>();
  face_size = hp_param[6];
  const float ratio = m.get("hp.patch_ratio").as<float>()[0];
  patch = (int)std::round(face_size * ratio);  // ForestParam::getPatchSize (Constants.hpp:27-30)
  n_forests = mp_param[7];
  ntrees_per_forest = mp_param[3];
  if (patch != 31) throw std::runtime_error("unsupported patch size (engine is built for 31x31 patches)");
  if (face_size > 125) throw std::runtime_error("unsupported face size (> 125)");
  for (const char* p : {"hp", "mp"}) {
    const auto& feats = m.get(std::string(p) + ".features");
    std::vector<int> f(feats.as<int32_t>(), feats.as<int32_t>() + feats.count());
    std::sort(f.begin(), f.end());
    if (f != std::vector<int>({0, 1, 2})) throw std::runtime_error("engine supports feature channels {0,1,2} only");
  }
  if (n_forests < 1 || n_forests > 5) throw std::runtime_error("engine supports 1..5 pose forests (poseT has 5 bins)");

  std::vector<uint4> nodes;
  std::vector<int32_t> roots, sizes;
  flatten_forest(m, "hp", nodes, roots, sizes);
  hp_trees = (int)roots.size();
  upload(hp_nodes, nodes, main_stream());
  hp_nodes_h = nodes;
  upload(hp_roots, roots, main_stream());
  hp_roots_h = roots;
  upload(hp_sizes, sizes, main_stream());
  flatten_forest(m, "mp", nodes, roots, sizes);
  if ((int)roots.size() != n_forests * ntrees_per_forest) throw std::runtime_error("FFD tree count mismatch");
  upload(mp_nodes, nodes, main_stream());
  mp_nodes_h = nodes;
  upload(mp_roots, roots, main_stream());
  mp_roots_h = roots;
  upload(mp_sizes, sizes, main_stream());
  HIP_CHECK(hipStreamSynchronize(main_stream()));  // host vectors are reused below

  // option-dependent leaf tables (head-pose values, FFD vote records) for desc's options
  hp_leaves = (int64_t)m.get("hp.leaf_n").count();
  mp_leaves = (int64_t)m.get("mp.leaf_n").count();
  for (int k = 0; k < 2; k++) {  // per tree: its leaf ordinals [off[t], off[t + 1]) (ffd_forest_tree_leaves)
    const std::string name = k ? "mp.tree_leaf_off" : "hp.tree_leaf_off";
    std::vector<int64_t>& v = k ? mp_tree_leaf_off : hp_tree_leaf_off;
    v.clear();
    if (m.has(name)) v.assign(m.get(name).as<int64_t>(), m.get(name).as<int64_t>() + m.get(name).count());
  }
  upload(hp_m, hp_leaf_values(m, desc.hp_option), main_stream());
  {
    VoteTable vt = mp_vote_records(m, desc.mp_option);
    vote_rec_compact = vt.compact;
    vote_bias_x = vt.bias_x;
    vote_bias_y = vt.bias_y;
    vote_range = vt.range;
    upload(mp_rec, vt.rec, main_stream());
  }
  load_cascade(m);
  HIP_CHECK(hipStreamSynchronize(main_stream()));
}

// head-pose leaf value m (face_utils.cpp:223-228): sum_j labels[j] * j over the option's labels,
// divided by (n * fg); -1 when the leaf fails the option's foreground test (it then casts no value).
std::vector<float> ffd_host::hp_leaf_values(const ffd::ModelFile& m, const ffd_headpose_option& o) {
  const auto& n = m.get("hp.leaf_n");
  const auto& fg = m.get("hp.leaf_fg");
  const auto& lb = m.get("hp.leaf_labels");
  const int64_t L = (int64_t)n.count();
  std::vector<float> mv(L);
  const int nl = std::max(0, std::min(o.num_head_pose_labels, (int)FFD_NUM_HP_LABELS));
  for (int64_t i = 0; i < L; i++) {
    const float f = fg.as<float>()[i];
    if (f > o.min_foreground_probability) {
      float v = 0;
      for (int j = 0; j < nl; j++) v += lb.as<int32_t>()[i * 5 + j] * j;
      v /= (n.as<int32_t>()[i] * f);
      mv[i] = v;
    } else {
      mv[i] = -1.f;
    }
  }
  return mv;
}

// FFD leaf vote records for k_votes: the filter of face_utils.cpp:276-290 under the option
// precomputed as a part mask, fg, and the offsets of the voting parts.  Compact 32-B records (offsets
// as u8 pairs relative to per-axis biases) when every voting offset fits, else 64-B records.
ffd_host::VoteTable ffd_host::mp_vote_records(const ffd::ModelFile& m, const ffd_multipart_option& op) {
  const auto& n = m.get("mp.leaf_n");
  const auto& fg = m.get("mp.leaf_fg");
  const auto& off = m.get("mp.leaf_offset");
  const auto& var = m.get("mp.leaf_var");
  const auto& pf = m.get("mp.leaf_pf");
  const int64_t leaves = (int64_t)n.count();
  const int np = std::max(0, std::min(op.num_parts, NPARTS));
  std::vector<uint32_t> mask(leaves);
  int mnx = 1 << 30, mny = 1 << 30, mxx = -(1 << 30), mxy = -(1 << 30);
  for (int64_t L = 0; L < leaves; L++) {
    uint32_t mk = 0;
    const float f = fg.as<float>()[L];
    for (int i = 0; i < np; i++) {
      float min_pf = op.min_pf;
      if (i == 0 || i == 7) min_pf *= 1.5;  // outer eye corners
      if (f > op.min_forground && pf.as<float>()[L * 10 + i] > min_pf && var.as<float>()[L * 10 + i] < op.max_variance &&
          n.as<int32_t>()[L] > op.min_samples) {
        mk |= 1u << i;
        const int x = off.as<int16_t>()[(L * 10 + i) * 2], y = off.as<int16_t>()[(L * 10 + i) * 2 + 1];
        mnx = std::min(mnx, x); mxx = std::max(mxx, x);
        mny = std::min(mny, y); mxy = std::max(mxy, y);
      }
    }
    mask[L] = mk;
  }
  VoteTable vt;
  vt.range.any = mnx <= mxx;
  if (vt.range.any) vt.range = VoteRange{true, mnx, mxx, mny, mxy};
  vt.compact = mxx - mnx <= 255 && mxy - mny <= 255;
  vt.bias_x = vt.compact && mnx <= mxx ? mnx : 0;
  vt.bias_y = vt.compact && mny <= mxy ? mny : 0;
  const int words = vt.compact ? 8 : 16;
  vt.rec.assign(leaves * words, 0);
  for (int64_t L = 0; L < leaves; L++) {
    uint32_t* r = &vt.rec[L * words];
    r[0] = mask[L];
    std::memcpy(&r[1], &fg.as<float>()[L], 4);
    for (int i = 0; i < NPARTS; i++) {
      const int x = off.as<int16_t>()[(L * 10 + i) * 2], y = off.as<int16_t>()[(L * 10 + i) * 2 + 1];
      if (vt.compact) {
        if (!((mask[L] >> i) & 1u)) continue;  // offsets of non-voting parts are never read
        const uint32_t u = (uint32_t)(x - vt.bias_x) | (uint32_t)(y - vt.bias_y) << 8;
        r[2 + i / 2] |= u << (16 * (i & 1));
      } else {
        r[2 + i] = (uint32_t)(uint16_t)x | (uint32_t)(uint16_t)y << 16;
      }
    }
  }
  return vt;
}

// The model's leaf payload arrays, read from the model file on first use (per-call estimator
// options, ffd_forest_leaves); the pipeline itself only uses the device tables.
const ffd::ModelFile& ffd_engine::leaf_arrays() {
  if (!leaf_model) {
    auto m = std::make_shared<ffd::ModelFile>();
    m->load(model_path, "leaf_");
    leaf_model = m;
  }
  return *leaf_model;
}

// Gabor coefficients: scale 0 = createKernel / initGaborKernels (FeatureChannelFactory.hpp:186-251)
// packed for k_gabor7; scales 1..4 = the separable factors of include/ffd_gabor.h packed for
// k_gabor_sep (block layout in ffd_kernels.hip).
void ffd_engine::build_gabor() {
  std::vector<float> coef(GABOR_COEF_TOTAL, 0.f);
  const double CV_PI = 3.1415926535897932384626433832795;
  const double sigma = 1.0 / 2.0 * CV_PI, dF = std::sqrt(2.0);
  {
    const int iNu = 0;
    std::vector<std::vector<float>> re(7), im(7);
    int Wk = 0;
    for (int iMu = 0; iMu < 7; iMu++) {
      double F = dF;
      double k = (CV_PI / 2) / std::pow(F, (double)iNu);
      double phi = CV_PI * iMu / 8;
      double width = std::round((sigma / k) * 6 + 1);
      if (std::fmod(width, 2.0) == 0.0) width++;
      Wk = (int)width;
      if (Wk != GABOR_WIDTHS[iNu]) throw std::runtime_error("unexpected Gabor kernel width");
      re[iMu].assign(Wk * Wk, 0.f);
      im[iMu].assign(Wk * Wk, 0.f);
      int off_set = (int)((width - 1) / 2);
      for (int i = 0; i < Wk; i++)
        for (int j = 0; j < Wk; j++) {
          int x = i - off_set, y = j - off_set;
          double dTemp1 = (std::pow(k, 2) / std::pow(sigma, 2)) *
                          std::exp(-(std::pow((double)x, 2) + std::pow((double)y, 2)) * std::pow(k, 2) /
                                   (2 * std::pow(sigma, 2)));
          double dTemp2 = std::cos(k * std::cos(phi) * x + k * std::sin(phi) * y) - std::exp(-(std::pow(sigma, 2) / 2));
          double dTemp3 = std::sin(k * std::cos(phi) * x + k * std::sin(phi) * y);
          re[iMu][j * Wk + i] = (float)(dTemp1 * dTemp2);
          im[iMu][j * Wk + i] = (float)(dTemp1 * dTemp3);
        }
    }
    for (int t = 0; t < 49; t++)  // interleaved (re, im) per orientation: one packed operand each
      for (int o = 0; o < 7; o++) {
        coef[GABOR_OFF0 + t * 16 + 2 * o] = re[o][t];
        coef[GABOR_OFF0 + t * 16 + 2 * o + 1] = im[o][t];
      }
  }
  for (int nu = 1; nu <= 4; nu++) {
    ffd_gabor_sep s;
    ffd_gabor_sep_init(nu, &s);
    const int R = s.R;
    if (2 * R + 1 != GABOR_WIDTHS[nu]) throw std::runtime_error("unexpected Gabor kernel width");
    float* b = coef.data() + GABOR_OFFS[nu];
    b[0] = s.c;
    float* v = b + 4;
    for (int t = 0; t <= R; t++) {
      v[12 * t] = s.g[t];
      for (int q = 0; q < 4; q++) {
        v[12 * t + 2 + 2 * q] = s.vc[q][t];
        v[12 * t + 3 + 2 * q] = s.vs[q][t];
      }
    }
    float* h = b + 4 + 12 * (R + 1);
    for (int t = -R; t <= R; t++) {
      const int at = t < 0 ? -t : t;
      auto hs = [&](int p) { return t < 0 ? -s.hs[p][at] : s.hs[p][at]; };
      float* e = h + 16 * (t + R);
      e[0] = s.hc[0][at]; e[1] = hs(0);
      e[2] = s.g[at]; e[3] = s.g[at];
      for (int p = 1; p <= 3; p++) {
        e[4 * p] = e[4 * p + 1] = s.hc[p][at];
        e[4 * p + 2] = e[4 * p + 3] = hs(p);
      }
    }
  }
  upload(gabor_coef, coef, main_stream());
  HIP_CHECK(hipStreamSynchronize(main_stream()));
}

// Run the whole pipeline for the chunk staged in w.h_fds (descriptor offsets are filled in
// here, relative to w's buffers).  Everything is enqueued on w.stream; nothing waits.
void ffd_engine::run_chunk(Workspace& w, const uint8_t* d_images, FaceOut* d_out) {
  std::vector<FaceDesc>& fds = w.h_fds;
  const int n = (int)fds.size();
  if (n == 0) return;
  const hipStream_t st = w.stream;
  int64_t gray_b = 0, mag_e = 0, ch_e = 0, hp_e = 0, mp_e = 0, vote_e = 0;
  // one channel plane stride for the whole batch (the traversal's window staging assumes it)
  int64_t plane = PITCH;
  int max_h = 1;
  int64_t max_src = 0;
  bool any_fint = false, any_wide = false;
  for (auto& f : fds)
    if (f.valid) {
      plane = std::max(plane, (int64_t)(f.H + 1) * PITCH);
      max_h = std::max(max_h, f.H);
      if (!f.nochan) max_src = std::max(max_src, (int64_t)f.bw * f.bh);
      any_fint |= f.fint != 0;
      f.wide = force_wide || votes_wide(f, desc.mp_option.step_size, mp_step_y(), patch / 2, vote_range);
      any_wide |= f.wide != 0;
    }
  for (auto& f : fds) {
    if (!f.valid) continue;
    f.gray_off = gray_b;
    gray_b += align_up((int64_t)f.H * PITCH, 256);
    f.mag_off = mag_e;
    mag_e += (int64_t)NGABOR * f.H * PITCH;
    f.plane = plane;
    f.ch_off = ch_e;
    ch_e += NCH * f.plane;
    f.hp_off = hp_e;
    hp_e += (int64_t)hp_trees * f.nhx * f.nhy;
    f.mp_off = mp_e;
    mp_e += (int64_t)MAX_TREES * f.nmx * f.nmy;
    f.vote_off = vote_e;  // (even: a wide face's VoteW records are 16-B aligned)
    vote_e += align_up((int64_t)NPARTS * MAX_TREES * f.nmx * f.nmy * (f.wide ? 2 : 1), 2);
  }
  w.gray.ensure(gray_b + 256);
  w.mag.ensure((mag_e + 64) * 4);
  w.chan.ensure((ch_e + 256) * 2);  // slack: traversal windows read up to 7 columns past a row
  w.hpleaf.ensure((hp_e + 64) * 4);
  w.mpleaf.ensure((mp_e + 64) * 4);
  w.votes.ensure((vote_e + 64) * sizeof(Vote));
  w.state.ensure((size_t)n * sizeof(HpState));
  w.ms_mean.ensure((size_t)n * NPARTS * 2 * 4);
  w.vote_counts.ensure((size_t)n * NPARTS * 4);
  w.ms_order.ensure((size_t)n * NPARTS * 4);
  w.gabor_redo.ensure((size_t)n * 5 * 4);  // 5 scales
  if (w.gabor_mm.n < (size_t)n * 5 * 64) {  // the banded instances leave their slots zeroed
    w.gabor_mm.ensure((size_t)n * 5 * 64);
    HIP_CHECK(hipMemsetAsync(w.gabor_mm.p, 0, w.gabor_mm.n, st));
  }
  upload_descriptors(w.faces, fds, st);
  HIP_CHECK(hipMemsetAsync(d_out, 0, (size_t)n * sizeof(FaceOut), st));

  const FaceDesc* dfd = w.faces.as<FaceDesc>();
  stage(0, st, [&] {
    launch_gray_resize(dfd, n, d_images, w.gray.as<uint8_t>(), st, max_src > (int64_t)1 << 30 ? 0 : (int)max_src);
  });
  // channel stage: Gabor scales 4..0 and the gray / Sobel integrals, dealt over the fork streams
  // (a large chunk fills the chip with one kernel at a time, so it forks only when FFD_CHANNEL_STREAMS
  // asks; a small one runs all six channel kernels side by side: single-face latency)
  const int nfork = n <= small_batch ? (int)w.fork.size() : std::min((int)w.fork.size(), channel_streams - 1);
  if (nfork > 0) {
    HIP_CHECK(hipEventRecord(w.fork_ev[0], st));
    for (int i = 0; i < nfork; i++) HIP_CHECK(hipStreamWaitEvent(w.fork[i], w.fork_ev[0], 0));
  }
  auto cs = [&](int i) { return i % (nfork + 1) == 0 ? st : w.fork[i % (nfork + 1) - 1]; };
  for (int nu = 4; nu >= 0; nu--) {  // largest kernels first
    const hipStream_t s2 = cs(4 - nu);
    stage(1 + (4 - nu), s2, [&] {
      launch_gabor(nu, dfd, n, max_h, w.gray.as<uint8_t>(), gabor_coef.as<float>(), w.mag.as<float>(),
                   w.chan.as<uint16_t>(), w.gabor_redo.as<int>(), gabor_exact, w.gabor_mm.as<uint32_t>(), s2);
    });
  }
  {
    const hipStream_t s2 = cs(5);
    stage(6, s2, [&] { launch_integral(dfd, n, max_h, w.gray.as<uint8_t>(), w.chan.as<uint16_t>(), s2); });
  }
  for (int i = 0; i < nfork; i++) {
    HIP_CHECK(hipEventRecord(w.fork_ev[1 + i], w.fork[i]));
    HIP_CHECK(hipStreamWaitEvent(st, w.fork_ev[1 + i], 0));
  }
  stage(7, st, [&] {
    launch_traverse(true, dfd, n, blocks_per_face(fds, true, trav_g_hp), trav_g_hp, hp_pairs.as<uint4>(),
                    hp_tops.as<uint4>(), hp_topi.as<uint32_t>(), trav_top_max, hp_far.as<uint32_t>(), nullptr,
                    hp_trees, desc.hp_option.step_size, desc.hp_option.step_size, plane, w.chan.as<uint16_t>(),
                    w.hpleaf.as<int32_t>(), trav_wg, TRAV_LDS_CAP, st);
    if (any_fint)
      launch_walk_fint(true, dfd, n, hp_nodes.as<uint4>(), hp_roots.as<int32_t>(), hp_trees, nullptr,
                       desc.hp_option.step_size, desc.hp_option.step_size, w.chan.as<uint16_t>(), w.hpleaf.as<int32_t>(), st);
  });
  stage(8, st, [&] {
    launch_hp_pose(dfd, n, w.hpleaf.as<int32_t>(), hp_m.as<float>(), hp_trees, n_forests, ntrees_per_forest,
                   w.state.as<HpState>(), d_out, st);
  });
  stage(9, st, [&] {
    launch_traverse(false, dfd, n, blocks_per_face(fds, false, trav_g_mp), trav_g_mp, mp_pairs.as<uint4>(),
                    mp_tops.as<uint4>(), mp_topi.as<uint32_t>(), trav_top_max, mp_far.as<uint32_t>(),
                    w.state.as<HpState>(), 0, desc.mp_option.step_size, mp_step_y(), plane, w.chan.as<uint16_t>(),
                    w.mpleaf.as<int32_t>(), trav_wg, TRAV_LDS_CAP, st);
    if (any_fint)
      launch_walk_fint(false, dfd, n, mp_nodes.as<uint4>(), mp_roots.as<int32_t>(), 0, w.state.as<HpState>(),
                       desc.mp_option.step_size, mp_step_y(), w.chan.as<uint16_t>(), w.mpleaf.as<int32_t>(), st);
  });
  const int n_parts = std::min(desc.mp_option.num_parts, NPARTS);
  stage(10, st, [&] {
    launch_votes(dfd, n, w.mpleaf.as<int32_t>(), mp_rec.as<uint4>(), vote_rec_compact, vote_bias_x, vote_bias_y,
                 w.state.as<HpState>(), MAX_TREES,
                 desc.mp_option.step_size, mp_step_y(), patch / 2, n_parts, w.votes.as<Vote>(), w.vote_counts.as<int32_t>(), st);
  });
  stage(11, st, [&] {
    launch_meanshift(dfd, n, w.state.as<HpState>(), MAX_TREES, n_parts, (float)desc.ms_option.kernel_size,
                     desc.ms_option.max_iterations, desc.ms_option.stopping_criteria, w.votes.as<Vote>(),
                     w.vote_counts.as<int32_t>(), w.ms_mean.as<float>(), d_out, w.ms_order.as<int32_t>(), st, any_wide);
  });
  HIP_CHECK(hipGetLastError());
}

// Split the batch into chunks, round-robin over the stream workspaces.  On return every chunk
// is enqueued and main_stream() is ordered after all of them.
// A chunk ends at max_chunk faces, where the faces change between ordinary and tall (H > MAX_FACE_H: a
// chunk has one channel plane stride, so a tall face would stretch its neighbours' planes), or before its
// buffers pass chunk_bytes (a few very tall faces).
void ffd_engine::analyze(const uint8_t* d_images, const std::vector<FaceDesc>& all, FaceOut* d_out) {
  const int n = (int)all.size();
  auto face_bytes = [&](const FaceDesc& f) -> int64_t {  // gray, mag, leaves, votes (VoteW past ~16 k rows)
    const int64_t pm = (int64_t)f.nmx * f.nmy;
    return (int64_t)f.H * PITCH * (1 + 4 * NGABOR) + 4 * ((int64_t)hp_trees * f.nhx * f.nhy + MAX_TREES * pm) +
           (int64_t)NPARTS * MAX_TREES * pm * sizeof(Vote) * (f.H > 16000 ? 2 : 1);
  };
  int k = 0;
  for (int first = 0; first < n; k++) {
    int cnt = 0, nvalid = 0, cls = -1;
    int64_t plane_max = PITCH, other = 0;
    while (first + cnt < n && cnt < max_chunk) {
      const FaceDesc& f = all[first + cnt];
      if (f.valid) {
        const int c = f.H > MAX_FACE_H;
        const int64_t pl = std::max(plane_max, (int64_t)(f.H + 1) * PITCH), o = other + face_bytes(f);
        if (nvalid > 0 && (c != cls || o + (int64_t)(nvalid + 1) * NCH * pl * 2 > chunk_bytes)) break;
        cls = c;
        plane_max = pl;
        other = o;
        nvalid++;
      }
      cnt++;
    }
    Workspace& w = *ws[k % ws.size()];
    // (h_fds reaches the device through a pinned staging slot that is reused only after its copy ran,
    // upload_descriptors; the device buffers are reused in stream order, so the host need not wait for
    // the workspace's last chunk)
    w.h_fds.assign(all.begin() + first, all.begin() + first + cnt);
    run_chunk(w, d_images, d_out + first);
    w.desc = w.h_fds;
    w.first = first;
    w.count = cnt;
    HIP_CHECK(hipEventRecord(w.done, w.stream));
    w.pending = true;
    last_ws = (int)(k % ws.size());
    first += cnt;
  }
  for (size_t i = 1; i < ws.size(); i++)
    if (ws[i]->pending) HIP_CHECK(hipStreamWaitEvent(main_stream(), ws[i]->done, 0));
}

ffd_status ffd_host::fail(ffd_engine* e, ffd_status s, const std::string& msg) {
  if (e) e->err = msg;
  else g_create_err = msg;
  return s;
}

// Fill the per-face descriptor (geometry + resize parameters) for a box on an image.  Returns the
// face's status: FFD_OK, FFD_ERR_INVALID_ARGUMENT (box outside the image or an empty scaled face:
// the reference's cv::Mat ROI / resize assertions throw) or FFD_ERR_OUT_OF_MEMORY (scaled face taller
// than MAX_FACE_ROWS: FFD_ERR_OUT_OF_MEMORY).  A face on which no head-pose patch fits runs like the reference: 0/0 head pose
// (NaN), trees 0..19 of forest 0, no votes, landmarks (0, 0); its channels are never read, so the
// channel stage skips it.
ffd_status ffd_host::make_desc(const ffd_engine* e, int64_t img_off, int iw, int ih, int stride, const ffd_rect& b,
                               FaceDesc& f) {
  std::memset(&f, 0, sizeof(f));
  f.img_off = img_off;
  f.img_w = iw; f.img_h = ih; f.img_stride = stride;
  f.bx = b.x; f.by = b.y; f.bw = b.width; f.bh = b.height;
  f.reject = FFD_ERR_INVALID_ARGUMENT;
  if (b.x < 0 || b.y < 0 || b.width <= 0 || b.height <= 0 || (int64_t)b.x + b.width > iw ||
      (int64_t)b.y + b.height > ih)
    return FFD_ERR_INVALID_ARGUMENT;
  Geometry g = e->geometry(b.width, b.height);
  if (g.W < 1 || g.H < 1 || g.W > PITCH - 3) return FFD_ERR_INVALID_ARGUMENT;
  if (g.H > MAX_FACE_ROWS) {  // > 50 GB of channel planes for this one face
    f.reject = FFD_ERR_OUT_OF_MEMORY;
    return FFD_ERR_OUT_OF_MEMORY;
  }
  if ((uint64_t)255 * g.W * g.H >= FINT_LIMIT) {  // float integrals past 2^31: rect_mean_fint is not exact there
    f.reject = FFD_ERR_UNSUPPORTED;
    return FFD_ERR_UNSUPPORTED;
  }
  f.W = g.W; f.H = g.H; f.scale = g.scale;
  f.fint = (int64_t)255 * g.W * g.H >= (int64_t)1 << 24 ? 1 : 0;  // an integral value may reach 2^24
  f.nhx = g.nhx; f.nhy = g.nhy; f.nmx = g.nmx; f.nmy = g.nmy;
  f.nochan = (f.nhx * f.nhy == 0 || g.W < 2 || g.H < 2) ? 1 : 0;
  if (g.W == b.width && g.H == b.height) {
    f.mode = 0;
  } else {
    double inv_x = (double)g.W / b.width, inv_y = (double)g.H / b.height;
    f.scale_x = 1. / inv_x;
    f.scale_y = 1. / inv_y;
    int ix = (int)std::nearbyint(f.scale_x), iy = (int)std::nearbyint(f.scale_y);
    bool area_fast = std::fabs(f.scale_x - ix) < DBL_EPSILON && std::fabs(f.scale_y - iy) < DBL_EPSILON;
    f.mode = (area_fast && ix == 2 && iy == 2) ? 2 : 1;
  }
  int xv = 0;
  while (xv <= g.W - 16) xv += 16;
  while (xv < g.W - 4) xv += 4;
  f.xv = xv;
  f.valid = 1;
  f.reject = FFD_OK;
  return FFD_OK;
}

namespace {

template <class F> ffd_status guarded(ffd_engine* e, F&& fn) {
  if (!e) return FFD_ERR_INVALID_ARGUMENT;
  try {
    HIP_CHECK(hipSetDevice(e->device));
    return fn();
  } catch (const DeviceOom& x) {
    return fail(e, FFD_ERR_OUT_OF_MEMORY, x.what());
  } catch (const Unsupported& x) {
    return fail(e, FFD_ERR_UNSUPPORTED, x.what());
  } catch (const HipError& x) {
    return fail(e, FFD_ERR_DEVICE, x.what());
  } catch (const std::bad_alloc&) {
    return fail(e, FFD_ERR_OUT_OF_MEMORY, "host allocation failed");
  } catch (const std::exception& x) {
    return fail(e, FFD_ERR_INTERNAL, x.what());
  }
}

}  // namespace

// Host images in, results in device memory (d_out, n_faces FaceOut), everything enqueued on the
// engine's streams; main_stream() is ordered after the batch on return.  Throws HipError.
// The images are uploaded on the engine's copy stream in host chunks of host_chunk faces, each chunk's
// new images (contiguous host runs coalesced into one copy) ahead of its compute, so the upload of
// chunk k + 1 overlaps the kernels of chunk k (SURVEY.md §8(d)'s H2D -> D2H timing rule, through the
// C ABI the C++ shim calls).
ffd_status ffd_host::analyze_host(ffd_engine* e, const ffd_image* imgs, int32_t n_img, const ffd_rect* boxes,
                                  const int32_t* box_img, int32_t n_faces, void* d_out) {
  if (n_faces < 0 || (n_faces > 0 && (!imgs || !boxes || !d_out)) || n_img < 0)
    return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
  if (!box_img && n_img != n_faces) return fail(e, FFD_ERR_INVALID_ARGUMENT, "box_img NULL requires n_img == n_faces");
  if (n_faces == 0) return FFD_OK;
  // device offsets: images packed back to back (the kernels read bytes), so host images that are
  // contiguous in memory stay contiguous and upload as one copy
  std::vector<int64_t> img_off(n_img);
  int64_t total = 0;
  for (int i = 0; i < n_img; i++) {
    if (!imgs[i].bgr || imgs[i].width <= 0 || imgs[i].height <= 0 || imgs[i].stride < 3 * imgs[i].width)
      return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad image " + std::to_string(i));
    img_off[i] = total;
    total += (int64_t)imgs[i].stride * imgs[i].height;
  }
  std::vector<FaceDesc> fds(n_faces);
  for (int i = 0; i < n_faces; i++) {
    int k = box_img ? box_img[i] : i;
    if (k < 0 || k >= n_img) return fail(e, FFD_ERR_INVALID_ARGUMENT, "box_img out of range");
    make_desc(e, img_off[k], imgs[k].width, imgs[k].height, imgs[k].stride, boxes[i], fds[i]);
  }
  e->sync_all();  // the staging buffer may still be read by the previous batch
  e->images.ensure(total + 16);
  uint8_t* dimg = e->images.as<uint8_t>();
  std::vector<char> sent(n_img, 0);
  const int hc = std::max(1, std::min(e->host_chunk, e->max_chunk));
  for (int lo = 0; lo < n_faces; lo += hc) {
    const int hi = std::min(n_faces, lo + hc);
    // this chunk's images not uploaded yet, in index order, coalesced into contiguous host runs
    std::vector<int> need;
    for (int i = lo; i < hi; i++) {
      const int k = box_img ? box_img[i] : i;
      if (!sent[k]) { sent[k] = 1; need.push_back(k); }
    }
    std::sort(need.begin(), need.end());
    for (size_t a = 0; a < need.size();) {
      size_t b = a + 1;
      int64_t bytes = (int64_t)imgs[need[a]].stride * imgs[need[a]].height;
      while (b < need.size() && need[b] == need[b - 1] + 1 &&
             imgs[need[b]].bgr == imgs[need[b - 1]].bgr + (int64_t)imgs[need[b - 1]].stride * imgs[need[b - 1]].height) {
        bytes += (int64_t)imgs[need[b]].stride * imgs[need[b]].height;
        b++;
      }
      HIP_CHECK(hipMemcpyAsync(dimg + img_off[need[a]], imgs[need[a]].bgr, (size_t)bytes, hipMemcpyHostToDevice,
                               e->copy_stream));
      a = b;
    }
    // every compute stream waits for the chunk's images
    HIP_CHECK(hipEventRecord(e->copy_done, e->copy_stream));
    for (auto& w : e->ws) HIP_CHECK(hipStreamWaitEvent(w->stream, e->copy_done, 0));
    std::vector<FaceDesc> part(fds.begin() + lo, fds.begin() + hi);
    e->analyze(dimg, part, static_cast<FaceOut*>(d_out) + lo);
  }
  return FFD_OK;
}

extern "C" {

const char* ffd_version(void) { return FFD_VERSION_STR; }

const char* ffd_status_string(int32_t s) {
  switch (s) {
    case FFD_OK: return "ok";
    case FFD_ERR_INVALID_ARGUMENT: return "invalid argument (face box outside the image or empty scaled face)";
    case FFD_ERR_MODEL: return "model file invalid or unsupported";
    case FFD_ERR_DEVICE: return "HIP device error or no HIP device";
    case FFD_ERR_OUT_OF_MEMORY: return "out of memory (or a scaled face over 2^21 rows)";
    case FFD_ERR_NOT_INITIALIZED: return "not initialised";
    case FFD_ERR_INTERNAL: return "internal error";
    case FFD_ERR_UNSUPPORTED: return "unsupported input (an image sample over 125 columns, or a detection frame over 2^18 raw candidates)";
    default: return "unknown status";
  }
}

void ffd_engine_desc_init(ffd_engine_desc* d) {
  if (!d) return;
  std::memset(d, 0, sizeof(*d));
  d->model_path = nullptr;
  d->device = 0;
  d->max_chunk_faces = 0;
  d->hp_option.num_head_pose_labels = 5;        // NUM_HEADPOSE_CLASSES
  d->hp_option.step_size = 4;
  d->hp_option.min_foreground_probability = 0.5f;
  d->mp_option.num_parts = 10;
  d->mp_option.step_size = 3;
  d->mp_option.min_samples = 2;
  d->mp_option.min_forground = 0.5f;
  d->mp_option.min_pf = 0.25f;
  d->mp_option.max_variance = 25.f;
  d->mp_option.step_size_y = 0;
  d->ms_option.kernel_size = 10;
  d->ms_option.max_iterations = 7;
  d->ms_option.stopping_criteria = 0.05f;
}

namespace {
// The engine's workspaces (streams, fork streams and their events) and the host-API copy stream.
void create_streams(ffd_engine* e) {
  for (int i = 0; i < std::max(1, e->n_streams); i++) {
    auto w = std::make_unique<Workspace>();
    HIP_CHECK(hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&w->done, hipEventDisableTiming));
    for (int j = 1; j < std::max(e->channel_streams, 6); j++) {
      hipStream_t f;
      HIP_CHECK(hipStreamCreateWithFlags(&f, hipStreamNonBlocking));
      w->fork.push_back(f);
    }
    for (int j = 0; j < std::max(e->channel_streams, 6); j++) {
      hipEvent_t ev;
      HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      w->fork_ev.push_back(ev);
    }
    e->ws.push_back(std::move(w));
  }
  HIP_CHECK(hipStreamCreateWithFlags(&e->copy_stream, hipStreamNonBlocking));
  HIP_CHECK(hipEventCreateWithFlags(&e->copy_done, hipEventDisableTiming));
}

ffd_status no_forests(ffd_engine* e) {
  return fail(e, FFD_ERR_INVALID_ARGUMENT, "a detector-only engine (ffd_detector_create) has no forests");
}
}  // namespace

ffd_status ffd_engine_create(const ffd_engine_desc* d, ffd_engine** out) {
  if (!out) return fail(nullptr, FFD_ERR_INVALID_ARGUMENT, "out is NULL");
  *out = nullptr;
  if (!d || !d->model_path) return fail(nullptr, FFD_ERR_INVALID_ARGUMENT, "desc/model_path is NULL");
  if (d->hp_option.step_size <= 0 || d->mp_option.step_size <= 0 || d->mp_option.step_size_y < 0 ||
      d->ms_option.kernel_size == 0)
    return fail(nullptr, FFD_ERR_INVALID_ARGUMENT, "invalid estimator options");
  std::unique_ptr<ffd_engine> e(new ffd_engine());
  e->desc = *d;
  e->device = d->device;
  auto shape = [](const char* v, TravShape& g) {  // "G" or "GXxGY"
    int x = 0, y = 0;
    if (std::sscanf(v, "%dx%d", &x, &y) == 2) g = TravShape{x, y};
    else if (std::sscanf(v, "%d", &x) == 1) g = TravShape{x, x};
  };
  if (const char* v = std::getenv("FFD_TRAV_G_HP")) shape(v, e->trav_g_hp);
  if (const char* v = std::getenv("FFD_TRAV_G_FFD")) shape(v, e->trav_g_mp);
  if (const char* v = std::getenv("FFD_TRAV_WG")) e->trav_wg = std::max(8, std::atoi(v));
  if (const char* v = std::getenv("FFD_TRAV_TOPMAX")) e->trav_top_max = std::max(1, std::min(TOP_CAP, std::atoi(v)));
  if (const char* v = std::getenv("FFD_VOTES_WIDE")) e->force_wide = std::atoi(v) != 0;
  if (const char* v = std::getenv("FFD_CHUNK_BYTES")) e->chunk_bytes = std::max<int64_t>(1, std::atoll(v));
  if (const char* v = std::getenv("FFD_GABOR_EXACT")) e->gabor_exact = std::atoi(v) != 0;
  if (const char* v = std::getenv("FFD_CHANNEL_STREAMS")) e->channel_streams = std::max(1, std::min(6, std::atoi(v)));
  if (const char* v = std::getenv("FFD_SMALL_BATCH")) e->small_batch = std::max(0, std::atoi(v));
  if (const char* v = std::getenv("FFD_HOST_CHUNK")) e->host_chunk = std::max(1, std::atoi(v));
  if (const char* v = std::getenv("FFD_CHUNK")) e->max_chunk = std::max(1, std::atoi(v));
  if (const char* v = std::getenv("FFD_STREAMS")) e->n_streams = std::max(1, std::min(8, std::atoi(v)));
  if (d->max_chunk_faces > 0) e->max_chunk = d->max_chunk_faces;
  try {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
      return fail(nullptr, FFD_ERR_DEVICE, "no HIP device available (the engine has no CPU fallback)");
    if (d->device < 0 || d->device >= ndev) return fail(nullptr, FFD_ERR_INVALID_ARGUMENT, "bad device ordinal");
    HIP_CHECK(hipSetDevice(d->device));
    create_streams(e.get());
    e->warm_descriptor_slots();
    e->model_path = d->model_path;
    e->load_model(d->model_path);
    e->check_traverse_lds();
    e->build_gabor();
  } catch (const HipError& x) {
    return fail(nullptr, FFD_ERR_DEVICE, x.what());
  } catch (const std::exception& x) {
    return fail(nullptr, FFD_ERR_MODEL, x.what());
  }
  *out = e.release();
  return FFD_OK;
}

// FaceForest::detectFace's CascadeClassifier (FaceForest.cpp:136-159, FaceForest.hpp:125-132) on its own: an
// engine that holds one Haar cascade, parsed from the OpenCV XML (the converter's reader), and no forests.
ffd_status ffd_detector_create(const char* cascade_xml, int32_t device, ffd_engine** out) {
  if (!out) return fail(nullptr, FFD_ERR_INVALID_ARGUMENT, "out is NULL");
  *out = nullptr;
  if (!cascade_xml || !*cascade_xml) return fail(nullptr, FFD_ERR_INVALID_ARGUMENT, "cascade_xml is empty");
  std::unique_ptr<ffd_engine> e(new ffd_engine());
  ffd_engine_desc_init(&e->desc);
  e->desc.device = device;
  e->device = device;
  e->detector_only = true;
  e->n_streams = 1;
  try {
    ffd::ModelFile m;
    ffd_host::cascade_arrays(cascade_xml, m);  // (a missing or malformed file fails here, as CascadeClassifier::load)
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
      return fail(nullptr, FFD_ERR_DEVICE, "no HIP device available (the engine has no CPU fallback)");
    if (device < 0 || device >= ndev) return fail(nullptr, FFD_ERR_INVALID_ARGUMENT, "bad device ordinal");
    HIP_CHECK(hipSetDevice(device));
    create_streams(e.get());
    e->warm_descriptor_slots();
    e->load_cascade(m);
    HIP_CHECK(hipStreamSynchronize(e->main_stream()));
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, device));
    e->n_cu = std::max(1, prop.multiProcessorCount);
  } catch (const HipError& x) {
    return fail(nullptr, FFD_ERR_DEVICE, x.what());
  } catch (const std::exception& x) {
    return fail(nullptr, FFD_ERR_MODEL, x.what());
  }
  *out = e.release();
  return FFD_OK;
}

void ffd_engine_destroy(ffd_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  release_comm(e);
  for (auto& w : e->ws) (void)hipStreamSynchronize(w->stream);
  e->orphan_samples();  // samples that outlive their engine keep only their host state
  delete e;
}

const char* ffd_last_error(const ffd_engine* e) { return e ? e->err.c_str() : g_create_err.c_str(); }

void* ffd_stream(ffd_engine* e) { return (e && !e->ws.empty()) ? (void*)e->main_stream() : nullptr; }

ffd_status ffd_synchronize(ffd_engine* e) {
  return guarded(e, [&] {
    e->sync_all();
    e->resolve();
    return FFD_OK;
  });
}

ffd_status ffd_check_mag_sqrt(ffd_engine* e, uint64_t* checked, uint64_t* mismatches) {
  return guarded(e, [&] {
    e->resolve();
    constexpr int kBlocks = 8192;
    const hipStream_t st = e->main_stream();
    e->scratch_c.ensure((size_t)kBlocks * 4 * 4);
    std::vector<uint32_t> bad((size_t)kBlocks * 4);
    uint64_t n_bad = 0, n_chk = 0;
    // mag_sqrt's exact domain: +0 and every finite s >= 2^-96 (bits 0x0F800000 .. 0x7F7FFFFF)
    const uint32_t ranges[2][2] = {{0u, 1u}, {0x0F800000u, 0x7F800000u - 0x0F800000u}};
    for (const auto& r : ranges) {
      launch_check_mag_sqrt(r[0], r[1], e->scratch_c.as<uint32_t>(), kBlocks, st);
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipMemcpyAsync(bad.data(), e->scratch_c.p, bad.size() * 4, hipMemcpyDeviceToHost, st));
      HIP_CHECK(hipStreamSynchronize(st));
      for (uint32_t b : bad) n_bad += b;
      n_chk += r[1];
    }
    if (checked) *checked = n_chk;
    if (mismatches) *mismatches = n_bad;
    return FFD_OK;
  });
}

static const char* const kStageNames[FFD_NUM_STAGES] = {
    "gray_resize", "gabor_25x25", "gabor_19x19", "gabor_13x13", "gabor_9x9", "gabor_7x7",
    "integral_channels", "headpose_traverse", "headpose_reduce_select", "ffd_traverse", "votes", "meanshift"};

const char* ffd_stage_name(int32_t i) { return (i >= 0 && i < FFD_NUM_STAGES) ? kStageNames[i] : ""; }

ffd_status ffd_set_profiling(ffd_engine* e, int32_t enable) {
  return guarded(e, [&] {
    e->resolve();
    e->profiling = enable != 0;
    for (int i = 0; i < FFD_NUM_STAGES; i++) { e->stage_ms[i] = 0; e->stage_n[i] = 0; }
    return FFD_OK;
  });
}

ffd_status ffd_get_stage_times(ffd_engine* e, double* ms, int64_t* launches, int32_t n) {
  return guarded(e, [&] {
    e->resolve();
    for (int i = 0; i < n && i < FFD_NUM_STAGES; i++) {
      if (ms) ms[i] = e->stage_ms[i];
      if (launches) launches[i] = e->stage_n[i];
    }
    return FFD_OK;
  });
}

ffd_status ffd_face_geometry(const ffd_engine* e, int32_t bw, int32_t bh, int32_t* fw, int32_t* fh, int32_t* nhp,
                             int32_t* nmp) {
  if (!e) return FFD_ERR_INVALID_ARGUMENT;
  Geometry g = e->geometry(bw, bh);
  if (g.W <= 0 || g.H <= 0) return FFD_ERR_INVALID_ARGUMENT;
  if (fw) *fw = g.W;
  if (fh) *fh = g.H;
  if (nhp) *nhp = g.nhx * g.nhy;
  if (nmp) *nmp = g.nmx * g.nmy;
  return FFD_OK;
}

ffd_status ffd_analyze_faces(ffd_engine* e, const ffd_image* imgs, int32_t n_img, const ffd_rect* boxes,
                             const int32_t* box_img, int32_t n_faces, ffd_face* out) {
  if (e && e->detector_only) return no_forests(e);
  return guarded(e, [&]() -> ffd_status {
    if (n_faces > 0 && !out) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    if (n_faces > 0) e->out.ensure((size_t)n_faces * sizeof(FaceOut));
    const ffd_status st = analyze_host(e, imgs, n_img, boxes, box_img, n_faces, e->out.p);
    if (st != FFD_OK || n_faces == 0) return st;
    static_assert(sizeof(FaceOut) == sizeof(ffd_face), "FaceOut must mirror ffd_face");
    HIP_CHECK(hipMemcpyAsync(out, e->out.p, (size_t)n_faces * sizeof(ffd_face), hipMemcpyDeviceToHost,
                             e->main_stream()));
    HIP_CHECK(hipStreamSynchronize(e->main_stream()));
    return FFD_OK;
  });
}

ffd_status ffd_analyze_faces_device(ffd_engine* e, const void* d_images, int64_t image_bytes, int32_t width,
                                    int32_t height, int32_t stride, int32_t n_img, const ffd_rect* boxes,
                                    const int32_t* box_img, int32_t n_faces, void* d_out) {
  if (e && e->detector_only) return no_forests(e);
  return guarded(e, [&]() -> ffd_status {
    if (n_faces < 0 || (n_faces > 0 && (!d_images || !boxes || !d_out)) || width <= 0 || height <= 0 ||
        stride < 3 * width || image_bytes < (int64_t)stride * height)
      return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    if (!box_img && n_img != n_faces) return fail(e, FFD_ERR_INVALID_ARGUMENT, "box_img NULL requires n_img == n_faces");
    std::vector<FaceDesc> fds(n_faces);
    for (int i = 0; i < n_faces; i++) {
      int k = box_img ? box_img[i] : i;
      if (k < 0 || k >= n_img) return fail(e, FFD_ERR_INVALID_ARGUMENT, "box_img out of range");
      make_desc(e, (int64_t)k * image_bytes, width, height, stride, boxes[i], fds[i]);
    }
    e->analyze(static_cast<const uint8_t*>(d_images), fds, static_cast<FaceOut*>(d_out));
    return FFD_OK;
  });
}

ffd_status ffd_get_trace(ffd_engine* e, int32_t index, ffd_trace* tr) {
  if (e && e->detector_only) return no_forests(e);
  return guarded(e, [&]() -> ffd_status {
    if (!tr) return fail(e, FFD_ERR_INVALID_ARGUMENT, "trace is NULL");
    if (e->last_ws < 0) return fail(e, FFD_ERR_INVALID_ARGUMENT, "no batch has run");
    Workspace& w = *e->ws[e->last_ws];
    const int k = index - w.first;
    if (k < 0 || k >= w.count) return fail(e, FFD_ERR_INVALID_ARGUMENT, "index not in the last chunk");
    const FaceDesc& f = w.desc[k];
    if (!f.valid) return fail(e, FFD_ERR_INVALID_ARGUMENT, "face was rejected");
    if (f.nochan && (tr->face || tr->channels))
      return fail(e, FFD_ERR_INVALID_ARGUMENT, "no head-pose patch fits this face: its channels were not computed");
    e->sync_all();
    const int W = f.W, H = f.H;
    if (tr->face)
      HIP_CHECK(hipMemcpy2D(tr->face, W, w.gray.as<uint8_t>() + f.gray_off, PITCH, W, H, hipMemcpyDeviceToHost));
    if (tr->channels) {
      std::vector<uint16_t> v((size_t)NCH * f.plane);
      HIP_CHECK(hipMemcpy(v.data(), w.chan.as<uint16_t>() + f.ch_off, v.size() * 2, hipMemcpyDeviceToHost));
      widen_integrals(v.data(), f.plane, W, H, tr->channels);
    }
    HpState hs;
    HIP_CHECK(hipMemcpy(&hs, w.state.as<HpState>() + k, sizeof(hs), hipMemcpyDeviceToHost));
    if (tr->hp_leaves) {
      const int nh = f.nhx * f.nhy;
      std::vector<int32_t> v((size_t)e->hp_trees * nh);
      HIP_CHECK(hipMemcpy(v.data(), w.hpleaf.as<int32_t>() + f.hp_off, v.size() * 4, hipMemcpyDeviceToHost));
      for (int xi = 0; xi < f.nhx; xi++)
        for (int yi = 0; yi < f.nhy; yi++)
          for (int t = 0; t < e->hp_trees; t++)
            tr->hp_leaves[(xi * f.nhy + yi) * e->hp_trees + t] = v[(size_t)(xi * f.nhy + yi) * e->hp_trees + t];
    }
    if (tr->mp_leaves) {
      const int nm = f.nmx * f.nmy, T = hs.n_trees;
      std::vector<int32_t> v((size_t)std::max(T, 1) * nm);
      HIP_CHECK(hipMemcpy(v.data(), w.mpleaf.as<int32_t>() + f.mp_off, (size_t)T * nm * 4, hipMemcpyDeviceToHost));
      for (int xi = 0; xi < f.nmx; xi++)
        for (int yi = 0; yi < f.nmy; yi++)
          for (int t = 0; t < T; t++) tr->mp_leaves[(xi * f.nmy + yi) * T + t] = v[(size_t)(xi * f.nmy + yi) * T + t];
    }
    if (tr->trees)
      for (int t = 0; t < MAX_TREES; t++) tr->trees[t] = t < hs.n_trees ? hs.trees[t] : -1;
    if (tr->pose_freq)
      for (int j = 0; j < 5; j++) tr->pose_freq[j] = j < e->n_forests ? hs.pose_freq[j] : 0.f;
    if (tr->vote_counts)
      HIP_CHECK(hipMemcpy(tr->vote_counts, w.vote_counts.as<int32_t>() + (size_t)k * NPARTS, NPARTS * 4,
                          hipMemcpyDeviceToHost));
    if (tr->ms_mean)
      HIP_CHECK(hipMemcpy(tr->ms_mean, w.ms_mean.as<float>() + (size_t)k * NPARTS * 2, NPARTS * 2 * 4,
                          hipMemcpyDeviceToHost));
    return FFD_OK;
  });
}

ffd_status ffd_extract_channels(ffd_engine* e, const uint8_t* gray_face, int32_t W, int32_t H, uint32_t* out) {
  if (e && e->detector_only) return no_forests(e);
  return guarded(e, [&]() -> ffd_status {
    if (!gray_face || !out || W < 2 || H < 2 || W > PITCH - 3 || H > MAX_FACE_ROWS)
      return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    // the face itself is the "image" (copy mode): one BGR image whose gray equals the input
    e->sync_all();
    Workspace& w = *e->ws[0];
    std::vector<uint8_t> bgr((size_t)W * H * 3);
    // BGR2GRAY of (v,v,v) is v: (1868+9617+4899)*v + 8192 >> 14 == v for v in [0,255]
    for (int i = 0; i < W * H; i++) bgr[3 * i] = bgr[3 * i + 1] = bgr[3 * i + 2] = gray_face[i];
    e->scratch_a.ensure(bgr.size());
    e->upload_pinned(e->scratch_a.p, bgr.data(), bgr.size(), w.stream);
    FaceDesc f;
    std::memset(&f, 0, sizeof(f));
    f.img_w = W; f.img_h = H; f.img_stride = 3 * W; f.bw = W; f.bh = H; f.W = W; f.H = H;
    f.fint = (int64_t)255 * W * H >= (int64_t)1 << 24 ? 1 : 0;  // OpenCV's float integral rounds past 2^24
    f.scale = 1.f; f.mode = 0; f.valid = 1;
    f.plane = (int64_t)(H + 1) * PITCH;
    w.gray.ensure((size_t)H * PITCH + 256);
    w.mag.ensure((size_t)NGABOR * H * PITCH * 4 + 256);
    w.chan.ensure((size_t)NCH * f.plane * 2 + 256);
    w.gabor_redo.ensure(5 * 4);
    if (w.gabor_mm.n < 5 * 64) {
      w.gabor_mm.ensure(5 * 64);
      HIP_CHECK(hipMemsetAsync(w.gabor_mm.p, 0, w.gabor_mm.n, w.stream));
    }
    std::vector<FaceDesc> one{f};
    upload(w.faces, one, w.stream);
    const FaceDesc* dfd = w.faces.as<FaceDesc>();
    launch_gray_resize(dfd, 1, e->scratch_a.as<uint8_t>(), w.gray.as<uint8_t>(), w.stream);
    for (int nu = 4; nu >= 0; nu--)
      launch_gabor(nu, dfd, 1, H, w.gray.as<uint8_t>(), e->gabor_coef.as<float>(), w.mag.as<float>(),
                   w.chan.as<uint16_t>(), w.gabor_redo.as<int>(), e->gabor_exact, w.gabor_mm.as<uint32_t>(), w.stream);
    launch_integral(dfd, 1, H, w.gray.as<uint8_t>(), w.chan.as<uint16_t>(), w.stream);
    HIP_CHECK(hipGetLastError());
    std::vector<uint16_t> v((size_t)NCH * f.plane);
    HIP_CHECK(hipMemcpyAsync(v.data(), w.chan.p, v.size() * 2, hipMemcpyDeviceToHost, w.stream));
    HIP_CHECK(hipStreamSynchronize(w.stream));
    widen_integrals(v.data(), f.plane, W, H, out);
    w.count = 0;  // workspace no longer holds a batch
    w.pending = false;
    if (e->last_ws == 0) e->last_ws = -1;
    return FFD_OK;
  });
}

}  // extern "C"

namespace {

// One image sample (38 integral planes, the reference's [c][H+1][W+1] layout) restricted to the
// region `r` as a one-face chunk on workspace 0: the region's integrals are the second differences
// of the sample's at the region origin (mod 2^16, exact for every rectangle a split reads), the
// patch grid covers the region (face_utils.cpp:197-207,255-265: x from bbox.x while
// x < bbox.x + bbox.width - patch) and votes keep sample coordinates (vox, voy).  The channel stage
// is skipped (nochan); the caller launches the forest stages.
void stage_desc(ffd_engine* e, Workspace& w, const FaceDesc& f);

// The descriptor of a sample region: patch grids over the region (face_utils.cpp:197-207,255-265: x from
// bbox.x while x < bbox.x + bbox.width - patch), votes in sample coordinates (vox, voy), channels staged.
FaceDesc region_desc(const ffd_engine* e, const ffd_rect& r, int hp_step, int mp_step_x, int mp_step_y) {
  FaceDesc f;
  std::memset(&f, 0, sizeof(f));
  const int rw = r.width, rh = r.height;
  const int P = e->patch;
  auto cnt = [&](int extent, int step) {
    int n = 0;
    for (int x = 0; x < extent - P; x += step) n++;
    return n;
  };
  f.W = rw; f.H = rh; f.bw = rw; f.bh = rh; f.scale = 1.f;
  f.nhx = cnt(rw, hp_step);
  f.nhy = cnt(rh, hp_step);
  f.nmx = cnt(rw, mp_step_x);
  f.nmy = cnt(rh, mp_step_y);
  f.vox = r.x; f.voy = r.y;
  f.valid = 1; f.nochan = 1;
  f.plane = (int64_t)(rh + 1) * PITCH;
  f.hp_off = f.mp_off = f.vote_off = f.ch_off = 0;
  return f;
}

FaceDesc stage_sample(ffd_engine* e, Workspace& w, const uint32_t* ch, int W, int H, const ffd_rect& r, int hp_step,
                      int mp_step_x, int mp_step_y) {
  FaceDesc f = region_desc(e, r, hp_step, mp_step_x, mp_step_y);
  const int rw = r.width, rh = r.height;
  std::vector<uint16_t> J((size_t)NCH * f.plane, 0);
  const size_t ow = (size_t)W + 1, oplane = ((size_t)H + 1) * ow;
  uint32_t vmax = 0;
  for (int c = 0; c < NCH; c++) {
    const uint32_t* I = ch + c * oplane;
    for (int y = 0; y <= rh; y++)
      for (int x = 0; x <= rw; x++) {
        const uint32_t v = I[(r.y + y) * ow + r.x + x];
        vmax = std::max(vmax, v);
        J[(size_t)c * f.plane + (size_t)y * PITCH + x] =
            (uint16_t)(v - I[r.y * ow + r.x + x] - I[(r.y + y) * ow + r.x] + I[r.y * ow + r.x]);
      }
  }
  if (vmax >= FINT_LIMIT) throw Unsupported("integral values of 2^31 or more (rect_mean_fint window)");
  f.fint = vmax >= (1u << 24) ? 1 : 0;  // float-rounded integrals (CV_32F past 2^24): k_walk_fint
  w.chan.ensure(J.size() * 2 + 512);  // slack: traversal windows read past a row
  HIP_CHECK(hipMemcpyAsync(w.chan.p, J.data(), J.size() * 2, hipMemcpyHostToDevice, w.stream));
  stage_desc(e, w, f);
  HIP_CHECK(hipStreamSynchronize(w.stream));  // J is released on return
  return f;
}

// The one-face descriptor of a staged sample region and the forest stages' buffers on workspace 0.
void stage_desc(ffd_engine* e, Workspace& w, const FaceDesc& f) {
  w.hpleaf.ensure(((size_t)e->hp_trees * f.nhx * f.nhy + 64) * 4);
  w.mpleaf.ensure(((size_t)MAX_TREES * f.nmx * f.nmy + 64) * 4);
  w.votes.ensure(((size_t)NPARTS * MAX_TREES * f.nmx * f.nmy + 64) * sizeof(Vote));
  w.state.ensure(sizeof(HpState));
  w.ms_mean.ensure(NPARTS * 2 * 4);
  w.vote_counts.ensure(NPARTS * 4);
  e->upload_descriptors(w.faces, std::vector<FaceDesc>{f}, w.stream);  // pinned staging: no synchronisation
  w.count = 0;  // the workspace no longer holds a batch for ffd_get_trace
  w.pending = false;
  if (e->last_ws == 0) e->last_ws = -1;
}

// Leaf tables for per-call estimator options: desc's own tables when the options match, else the
// tables built for the last differing options (rebuilt when they change).
bool same(const ffd_headpose_option& a, const ffd_headpose_option& b) {
  return a.num_head_pose_labels == b.num_head_pose_labels &&
         a.min_foreground_probability == b.min_foreground_probability;
}
bool same(const ffd_multipart_option& a, const ffd_multipart_option& b) {
  return a.num_parts == b.num_parts && a.min_samples == b.min_samples && a.min_forground == b.min_forground &&
         a.min_pf == b.min_pf && a.max_variance == b.max_variance;
}
const float* hp_table(ffd_engine* e, const ffd_headpose_option& o) {
  if (same(o, e->desc.hp_option)) return e->hp_m.as<float>();
  if (!e->alt.hp_ok || !same(o, e->alt.hp)) {
    e->sync_all();
    upload(e->alt.hp_m, hp_leaf_values(e->leaf_arrays(), o), e->main_stream());
    HIP_CHECK(hipStreamSynchronize(e->main_stream()));
    e->alt.hp = o;
    e->alt.hp_ok = true;
  }
  return e->alt.hp_m.as<float>();
}
const uint4* mp_table(ffd_engine* e, const ffd_multipart_option& o, bool& compact, int& bx, int& by, VoteRange& vr) {
  if (same(o, e->desc.mp_option)) {
    compact = e->vote_rec_compact; bx = e->vote_bias_x; by = e->vote_bias_y; vr = e->vote_range;
    return e->mp_rec.as<uint4>();
  }
  if (!e->alt.mp_ok || !same(o, e->alt.mp)) {
    e->sync_all();
    VoteTable vt = mp_vote_records(e->leaf_arrays(), o);
    upload(e->alt.mp_rec, vt.rec, e->main_stream());
    HIP_CHECK(hipStreamSynchronize(e->main_stream()));
    e->alt.compact = vt.compact; e->alt.bias_x = vt.bias_x; e->alt.bias_y = vt.bias_y; e->alt.range = vt.range;
    e->alt.mp = o;
    e->alt.mp_ok = true;
  }
  compact = e->alt.compact; bx = e->alt.bias_x; by = e->alt.bias_y; vr = e->alt.range;
  return e->alt.mp_rec.as<uint4>();
}

bool region_ok(int W, int H, const ffd_rect* r) {
  return r && r->x >= 0 && r->y >= 0 && r->width > 0 && r->height > 0 && (int64_t)r->x + r->width <= W &&
         (int64_t)r->y + r->height <= H && r->width <= PITCH - 3 && r->height <= MAX_FACE_ROWS;
}

// getHeadPoseVotesMT + the pose reduction (FaceForest.cpp:60-72, face_utils.cpp:183-242) on the staged
// one-face chunk f of workspace w whose planes are `chan`.
HpState run_headpose(ffd_engine* e, Workspace& w, const FaceDesc& f, const uint16_t* chan, const ffd_headpose_option& o) {
  const float* hp_m = hp_table(e, o);
  const TravShape g = ffd_engine::fit_shape(e->trav_g_hp, true, o.step_size, o.step_size);
  const FaceDesc* dfd = w.faces.as<FaceDesc>();
  std::vector<FaceDesc> fv{f};
  e->out.ensure(sizeof(FaceOut));
  launch_traverse(true, dfd, 1, blocks_per_face(fv, true, g), g, e->hp_pairs.as<uint4>(), e->hp_tops.as<uint4>(),
                  e->hp_topi.as<uint32_t>(), e->trav_top_max, e->hp_far.as<uint32_t>(), nullptr, e->hp_trees,
                  o.step_size, o.step_size, f.plane, chan, w.hpleaf.as<int32_t>(), e->trav_wg, TRAV_LDS_CAP, w.stream);
  if (f.fint)
    launch_walk_fint(true, dfd, 1, e->hp_nodes.as<uint4>(), e->hp_roots.as<int32_t>(), e->hp_trees, nullptr, o.step_size,
                     o.step_size, chan, w.hpleaf.as<int32_t>(), w.stream);
  launch_hp_pose(dfd, 1, w.hpleaf.as<int32_t>(), hp_m, e->hp_trees, e->n_forests, e->ntrees_per_forest,
                 w.state.as<HpState>(), e->out.as<FaceOut>(), w.stream);
  HIP_CHECK(hipGetLastError());
  HpState hs;
  HIP_CHECK(hipMemcpyAsync(&hs, w.state.p, sizeof(hs), hipMemcpyDeviceToHost, w.stream));
  HIP_CHECK(hipStreamSynchronize(w.stream));
  return hs;
}

ffd_status check_mp_call(ffd_engine* e, const int32_t* tree_ids, int n_trees, const ffd_multipart_option& o) {
  if (n_trees < 1 || n_trees > MAX_TREES || !tree_ids) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
  const int ntot = e->n_forests * e->ntrees_per_forest;
  for (int t = 0; t < n_trees; t++)
    if (tree_ids[t] < 0 || tree_ids[t] >= ntot) return fail(e, FFD_ERR_INVALID_ARGUMENT, "tree id out of range");
  if (o.step_size <= 0 || o.step_size_y < 0) return fail(e, FFD_ERR_INVALID_ARGUMENT, "invalid MultiPartEstimatorOption");
  return FFD_OK;
}

// getFacialFeaturesVotesMT + MeanShift (FaceForest.cpp:74-95, face_utils.cpp:244-302) on the staged one-face
// chunk f of workspace w (planes `chan`) with the given trees; points in sample coordinates.
void run_facial_features(ffd_engine* e, Workspace& w, FaceDesc f, const uint16_t* chan, const int32_t* tree_ids,
                         int n_trees, const ffd_multipart_option& o, int32_t* points) {
  const int step_y = o.step_size_y > 0 ? o.step_size_y : o.step_size;
  bool compact = false;
  int bias_x = 0, bias_y = 0;
  VoteRange vr;
  const uint4* rec = mp_table(e, o, compact, bias_x, bias_y, vr);
  f.wide = e->force_wide || votes_wide(f, o.step_size, step_y, e->patch / 2, vr);
  if (f.wide) {  // VoteW lists: twice the vote space, and the descriptor again
    w.votes.ensure(((size_t)2 * NPARTS * MAX_TREES * f.nmx * f.nmy + 64) * sizeof(Vote));
    e->upload_descriptors(w.faces, std::vector<FaceDesc>{f}, w.stream);
  }
  const TravShape g = ffd_engine::fit_shape(e->trav_g_mp, false, o.step_size, step_y);
  const FaceDesc* dfd = w.faces.as<FaceDesc>();
  std::vector<FaceDesc> fv{f};
  HpState hs;
  std::memset(&hs, 0, sizeof(hs));
  hs.n_trees = n_trees;
  for (int t = 0; t < n_trees; t++) hs.trees[t] = tree_ids[t];
  e->upload_pinned(w.state.p, &hs, sizeof(hs), w.stream);
  e->out.ensure(sizeof(FaceOut));
  const int n_parts = std::max(0, std::min(o.num_parts, NPARTS));
  launch_traverse(false, dfd, 1, blocks_per_face(fv, false, g), g, e->mp_pairs.as<uint4>(), e->mp_tops.as<uint4>(),
                  e->mp_topi.as<uint32_t>(), e->trav_top_max, e->mp_far.as<uint32_t>(), w.state.as<HpState>(), 0,
                  o.step_size, step_y, f.plane, chan, w.mpleaf.as<int32_t>(), e->trav_wg, TRAV_LDS_CAP, w.stream);
  if (f.fint)
    launch_walk_fint(false, dfd, 1, e->mp_nodes.as<uint4>(), e->mp_roots.as<int32_t>(), 0, w.state.as<HpState>(),
                     o.step_size, step_y, chan, w.mpleaf.as<int32_t>(), w.stream);
  launch_votes(dfd, 1, w.mpleaf.as<int32_t>(), rec, compact, bias_x, bias_y, w.state.as<HpState>(), MAX_TREES,
               o.step_size, step_y, e->patch / 2, n_parts, w.votes.as<Vote>(), w.vote_counts.as<int32_t>(), w.stream);
  // FaceForest::estimateFacialFeatures shifts with a default MeanShiftOption (FaceForest.cpp:89-92)
  launch_meanshift(dfd, 1, w.state.as<HpState>(), MAX_TREES, n_parts, 10.f, 7, 0.05f, w.votes.as<Vote>(),
                   w.vote_counts.as<int32_t>(), w.ms_mean.as<float>(), e->out.as<FaceOut>(), nullptr, w.stream, f.wide != 0);
  HIP_CHECK(hipGetLastError());
  FaceOut out;
  HIP_CHECK(hipMemcpyAsync(&out, e->out.p, sizeof(out), hipMemcpyDeviceToHost, w.stream));
  HIP_CHECK(hipStreamSynchronize(w.stream));
  for (int i = 0; i < NPARTS; i++) {  // scale 1: cvRound of the MeanShift mode, sample coordinates
    points[2 * i] = i < n_parts ? out.points[i][0] : 0;
    points[2 * i + 1] = i < n_parts ? out.points[i][1] : 0;
  }
}

}  // namespace

extern "C" {

ffd_status ffd_estimate_headpose(ffd_engine* e, const uint32_t* channels, int32_t W, int32_t H,
                                 const ffd_rect* region, const ffd_headpose_option* options, float* headpose,
                                 float* variance) {
  if (e && e->detector_only) return no_forests(e);
  return guarded(e, [&]() -> ffd_status {
    if (!channels || W < 1 || H < 1) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    const ffd_rect full{0, 0, W, H};
    if (!region) region = &full;
    if (!region_ok(W, H, region)) return fail(e, FFD_ERR_INVALID_ARGUMENT, "face_bbox outside the image sample");
    const ffd_headpose_option o = options ? *options : e->desc.hp_option;
    if (o.step_size <= 0) return fail(e, FFD_ERR_INVALID_ARGUMENT, "invalid HeadPoseEstimatorOption");
    e->sync_all();
    Workspace& w = *e->ws[0];
    const FaceDesc f = stage_sample(e, w, channels, W, H, *region, o.step_size, e->desc.mp_option.step_size,
                                    e->mp_step_y());
    const HpState hs = run_headpose(e, w, f, w.chan.as<uint16_t>(), o);
    if (headpose) *headpose = hs.headpose;
    if (variance) *variance = hs.variance;
    return FFD_OK;
  });
}

ffd_status ffd_estimate_facial_features(ffd_engine* e, const uint32_t* channels, int32_t W, int32_t H,
                                        const ffd_rect* region, const int32_t* tree_ids, int32_t n_trees,
                                        const ffd_multipart_option* options, int32_t* points) {
  if (e && e->detector_only) return no_forests(e);
  return guarded(e, [&]() -> ffd_status {
    if (!channels || !points || W < 1 || H < 1) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    const ffd_rect full{0, 0, W, H};
    if (!region) region = &full;
    if (!region_ok(W, H, region)) return fail(e, FFD_ERR_INVALID_ARGUMENT, "face_bbox outside the image sample");
    const ffd_multipart_option o = options ? *options : e->desc.mp_option;
    const ffd_status st = check_mp_call(e, tree_ids, n_trees, o);
    if (st != FFD_OK) return st;
    const int step_y = o.step_size_y > 0 ? o.step_size_y : o.step_size;
    e->sync_all();
    Workspace& w = *e->ws[0];
    const FaceDesc f = stage_sample(e, w, channels, W, H, *region, e->desc.hp_option.step_size, o.step_size, step_y);
    run_facial_features(e, w, f, w.chan.as<uint16_t>(), tree_ids, n_trees, o, points);
    return FFD_OK;
  });
}

ffd_status ffd_forest_tree_leaves(ffd_engine* e, int32_t kind, int32_t tree_id, int32_t* first, int32_t* count) {
  if (e && e->detector_only) return no_forests(e);
  return guarded(e, [&]() -> ffd_status {
    if (!first || !count) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    if (kind != FFD_FOREST_HEADPOSE && kind != FFD_FOREST_FFD) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad forest kind");
    const std::vector<int64_t>& off = kind == FFD_FOREST_HEADPOSE ? e->hp_tree_leaf_off : e->mp_tree_leaf_off;
    if (tree_id < 0 || (size_t)tree_id + 1 >= off.size()) return fail(e, FFD_ERR_INVALID_ARGUMENT, "tree id out of range");
    *first = (int32_t)off[tree_id];
    *count = (int32_t)(off[tree_id + 1] - off[tree_id]);
    return FFD_OK;
  });
}

ffd_status ffd_forest_leaves(ffd_engine* e, int32_t kind, const int32_t* leaf_ids, int32_t n, void* out) {
  if (e && e->detector_only) return no_forests(e);
  return guarded(e, [&]() -> ffd_status {
    if ((n > 0 && (!leaf_ids || !out)) || n < 0) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    if (kind != FFD_FOREST_HEADPOSE && kind != FFD_FOREST_FFD) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad forest kind");
    const int64_t L = kind == FFD_FOREST_HEADPOSE ? e->hp_leaves : e->mp_leaves;
    for (int i = 0; i < n; i++)
      if (leaf_ids[i] < 0 || leaf_ids[i] >= L) return fail(e, FFD_ERR_INVALID_ARGUMENT, "leaf ordinal out of range");
    if (n == 0) return FFD_OK;
    const ffd::ModelFile& m = e->leaf_arrays();
    if (kind == FFD_FOREST_HEADPOSE) {  // HeadPoseLeaf (HeadPoseSample.hpp:144-162)
      const int32_t* ln = m.get("hp.leaf_n").as<int32_t>();
      const float* fg = m.get("hp.leaf_fg").as<float>();
      const int32_t* lb = m.get("hp.leaf_labels").as<int32_t>();
      ffd_headpose_leaf* o = static_cast<ffd_headpose_leaf*>(out);
      for (int i = 0; i < n; i++) {
        const int64_t k = leaf_ids[i];
        o[i].hp_nsamples = ln[k];
        o[i].hp_foreground = fg[k];
        for (int j = 0; j < FFD_NUM_HP_LABELS; j++) o[i].hp_labels[j] = lb[k * FFD_NUM_HP_LABELS + j];
      }
    } else {  // MPLeaf (MPSample.hpp:137-159)
      const int32_t* ln = m.get("mp.leaf_n").as<int32_t>();
      const float* fg = m.get("mp.leaf_fg").as<float>();
      const int16_t* off = m.get("mp.leaf_offset").as<int16_t>();
      const float* var = m.get("mp.leaf_var").as<float>();
      const float* pf = m.get("mp.leaf_pf").as<float>();
      ffd_mp_leaf* o = static_cast<ffd_mp_leaf*>(out);
      for (int i = 0; i < n; i++) {
        const int64_t k = leaf_ids[i];
        o[i].mp_samples = ln[k];
        o[i].mp_foreground = fg[k];
        for (int j = 0; j < FFD_NUM_LANDMARKS; j++) {
          o[i].mp_parts_offset[j][0] = off[(k * 10 + j) * 2];
          o[i].mp_parts_offset[j][1] = off[(k * 10 + j) * 2 + 1];
          o[i].mp_parts_variance[j] = var[k * 10 + j];
          o[i].mp_prob_foreground[j] = pf[k * 10 + j];
        }
      }
    }
    return FFD_OK;
  });
}

ffd_status ffd_forest_eval_leaves(ffd_engine* e, int32_t kind, const uint32_t* channels, int32_t W, int32_t H,
                                  const int32_t* patches_xy, int32_t n_patches, const int32_t* tree_ids, int32_t n_trees,
                                  int32_t* leaf_ids) {
  if (e && e->detector_only) return no_forests(e);
  return guarded(e, [&]() -> ffd_status {
    if (!channels || (!patches_xy && n_patches) || (!tree_ids && n_trees) || (!leaf_ids && (int64_t)n_patches * n_trees) ||
        W < 1 || H < 1 || W > PITCH - 3 || H > MAX_FACE_ROWS || n_patches < 0 || n_trees < 0)
      return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    if (kind != FFD_FOREST_HEADPOSE && kind != FFD_FOREST_FFD) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad forest kind");
    const int ntot = kind == FFD_FOREST_HEADPOSE ? e->hp_trees : e->n_forests * e->ntrees_per_forest;
    for (int t = 0; t < n_trees; t++)
      if (tree_ids[t] < 0 || tree_ids[t] >= ntot) return fail(e, FFD_ERR_INVALID_ARGUMENT, "tree id out of range");
    for (int p = 0; p < n_patches; p++) {
      const int x = patches_xy[2 * p], y = patches_xy[2 * p + 1];
      if (x < 0 || y < 0 || x + e->patch > W || y + e->patch > H)
        return fail(e, FFD_ERR_INVALID_ARGUMENT, "patch outside the image sample");
    }
    if (n_patches == 0 || n_trees == 0) return FFD_OK;
    if ((int64_t)n_patches * n_trees >= ((int64_t)1 << 31))  // k_eval_patches indexes (patch, tree) in int
      return fail(e, FFD_ERR_UNSUPPORTED, "patches x trees of 2^31 or more");
    const int64_t plane = (int64_t)(H + 1) * PITCH;
    // the device keeps integrals modulo 2^16 (exact for every rectangle the trees read)
    std::vector<uint16_t> narrow((size_t)NCH * plane, 0);
    uint32_t vmax = 0;
    for (int c = 0; c < NCH; c++)
      for (int y = 0; y <= H; y++)
        for (int x = 0; x <= W; x++) {
          const uint32_t v = channels[((size_t)c * (H + 1) + y) * (W + 1) + x];
          vmax = std::max(vmax, v);
          narrow[(size_t)c * plane + (size_t)y * PITCH + x] = (uint16_t)v;
        }
    if (vmax >= FINT_LIMIT) return fail(e, FFD_ERR_UNSUPPORTED, "integral values of 2^31 or more (rect_mean_fint window)");
    upload(e->scratch_a, narrow, e->main_stream());
    std::vector<int32_t> pv(patches_xy, patches_xy + 2 * n_patches), tv(tree_ids, tree_ids + n_trees);
    upload(e->scratch_b, pv, e->main_stream());
    upload(e->scratch_c, tv, e->main_stream());
    DevBuf outb;
    outb.ensure((size_t)n_patches * n_trees * 4);
    const bool hp = kind == FFD_FOREST_HEADPOSE;
    launch_eval_patches(hp ? e->hp_nodes.as<uint4>() : e->mp_nodes.as<uint4>(),
                        hp ? e->hp_roots.as<int32_t>() : e->mp_roots.as<int32_t>(), e->scratch_c.as<int32_t>(), n_trees,
                        e->scratch_b.as<int32_t>(), n_patches, e->scratch_a.as<uint16_t>(), plane, outb.as<int32_t>(),
                        e->main_stream(), vmax >= (1u << 24));  // float-rounded integrals: rect_mean_fint
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(leaf_ids, outb.p, (size_t)n_patches * n_trees * 4, hipMemcpyDeviceToHost, e->main_stream()));
    HIP_CHECK(hipStreamSynchronize(e->main_stream()));  // `narrow` outlives the upload
    return FFD_OK;
  });
}

}  // extern "C"

// ------------------------------------------------------------------ image samples --
// ImageSample kept on the device (ffd.h "Device-resident image samples").
struct ffd_sample {
  ffd_engine* e = nullptr;  // nullptr once the engine was destroyed first (the sample is then orphaned)
  int device = 0;
  int W = 0, H = 0;
  int64_t plane = 0;  // (H + 1) * PITCH
  int fint = 0;       // float-rounded integrals (CV_32F past 2^24, FaceDesc::fint): walked by rect_mean_fint
  DevBuf chan;        // u16 [NCH][H + 1][PITCH], integrals mod 2^16
  DevBuf desc;        // the grid traversal's one-face descriptor, kept for the steps it was made for
  int desc_hp = -1, desc_mp = -1;
};

void ffd_engine::orphan_samples() {
  std::lock_guard<std::mutex> g(samples_mu);
  for (ffd_sample* s : samples) {
    if (s->chan.p) (void)hipFree(s->chan.p);
    s->chan.p = nullptr;
    s->chan.n = 0;
    if (s->desc.p) (void)hipFree(s->desc.p);
    s->desc.p = nullptr;
    s->desc.n = 0;
    s->e = nullptr;
  }
  samples.clear();
}

namespace {

// A sample's channel planes as a one-face chunk of workspace 0 (region = the whole sample).
FaceDesc sample_desc(ffd_sample* s, int hp_step, int mp_step_x, int mp_step_y) {
  const ffd_rect full{0, 0, s->W, s->H};
  FaceDesc f = region_desc(s->e, full, hp_step, mp_step_x, mp_step_y);
  f.plane = s->plane;
  f.fint = s->fint;
  return f;
}

// The sample's one-face descriptor for the grid traversal (head-pose step khp, FFD step kmp on both axes), kept on
// the device with the sample and uploaded again only for other steps.
const FaceDesc* grid_desc(ffd_engine* e, ffd_sample* s, int khp, int kmp, hipStream_t st) {
  if (s->desc_hp != khp || s->desc_mp != kmp || !s->desc.p) {
    const FaceDesc f = sample_desc(s, khp, kmp, kmp);
    s->desc.ensure(sizeof(FaceDesc));
    e->upload_pinned(s->desc.p, &f, sizeof(f), st);
    s->desc_hp = khp;
    s->desc_mp = kmp;
  }
  return s->desc.as<FaceDesc>();
}

ffd_status orphaned() {
  return fail(nullptr, FFD_ERR_INVALID_ARGUMENT, "the image sample's engine was destroyed (ffd_engine_destroy ran first)");
}

bool sample_size_ok(int W, int H) {
  return W >= 2 && H >= 2 && W <= PITCH - 3 && H <= MAX_FACE_ROWS && (uint64_t)255 * W * H < FINT_LIMIT;
}

ffd_status sample_eval(ffd_sample* s, int32_t kind, const int32_t* patches_xy, int32_t n_patches, int x0, int y0,
                       int step, int nx, int ny, const int32_t* tree_ids, int32_t n_trees, int32_t* leaf_ids) {
  ffd_engine* e = s->e;
  const bool grid = patches_xy == nullptr;
  if (kind != FFD_FOREST_HEADPOSE && kind != FFD_FOREST_FFD) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad forest kind");
  if (n_trees < 0 || n_trees > MAX_TREES || (n_trees && !tree_ids) || n_patches < 0)
    return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
  const int ntot = kind == FFD_FOREST_HEADPOSE ? e->hp_trees : e->n_forests * e->ntrees_per_forest;
  for (int t = 0; t < n_trees; t++)
    if (tree_ids[t] < 0 || tree_ids[t] >= ntot) return fail(e, FFD_ERR_INVALID_ARGUMENT, "tree id out of range");
  const int P = e->patch;
  if (grid) {
    if (nx < 0 || ny < 0 || (nx && ny && (step <= 0 || x0 < 0 || y0 < 0 || x0 + (int64_t)(nx - 1) * step + P > s->W ||
                                          y0 + (int64_t)(ny - 1) * step + P > s->H)))
      return fail(e, FFD_ERR_INVALID_ARGUMENT, "patch grid outside the image sample");
    if ((int64_t)nx * ny * std::max(n_trees, 1) >= ((int64_t)1 << 31))  // k_sample_eval indexes (patch, tree) in int
      return fail(e, FFD_ERR_UNSUPPORTED, "patch grid x trees of 2^31 or more");
    n_patches = nx * ny;
  } else {
    for (int p = 0; p < n_patches; p++) {
      const int x = patches_xy[2 * p], y = patches_xy[2 * p + 1];
      if (x < 0 || y < 0 || x + P > s->W || y + P > s->H)
        return fail(e, FFD_ERR_INVALID_ARGUMENT, "patch outside the image sample");
    }
  }
  if (n_patches == 0 || n_trees == 0) return FFD_OK;
  if (!leaf_ids) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
  if ((int64_t)n_patches * n_trees >= ((int64_t)1 << 31)) return fail(e, FFD_ERR_UNSUPPORTED, "patches x trees of 2^31 or more");
  const bool hp = kind == FFD_FOREST_HEADPOSE;
  // A grid from the origin with the estimators' rule (face_utils.cpp:197-207,255-265) runs as the batch path's
  // traversal of a one-face chunk (k_traverse: LDS windows, tree tops, pair records), which writes the leaves in
  // exactly the grid order; the grid asked for is a leading sub-grid of it.
  bool all_hp_trees = hp && n_trees == e->hp_trees;
  for (int t = 0; all_hp_trees && t < n_trees; t++) all_hp_trees = tree_ids[t] == t;
  if (grid && x0 == 0 && y0 == 0 && (!hp || all_hp_trees) && step <= 32 && n_trees <= MAX_TREES && !s->fint) {
    const int khp = hp ? step : e->desc.hp_option.step_size, kmp = hp ? e->desc.mp_option.step_size : step;
    const FaceDesc f = sample_desc(s, khp, kmp, kmp);
    const int gx = hp ? f.nhx : f.nmx, gy = hp ? f.nhy : f.nmy;
    if (nx <= gx && ny <= gy) {
      e->sync_all();
      Workspace& w = *e->ws[0];
      w.count = 0;  // the workspace no longer holds a batch for ffd_get_trace
      w.pending = false;
      if (e->last_ws == 0) e->last_ws = -1;
      const TravShape g = ffd_engine::fit_shape(hp ? e->trav_g_hp : e->trav_g_mp, hp, step, step);
      std::vector<FaceDesc> fv{f};
      // the leaves go straight to host-mapped pinned memory (no device buffer, no copy back)
      const size_t all = (size_t)gx * gy * n_trees * 4;
      int32_t* pin = static_cast<int32_t*>(e->pin_leaf.ensure(all));
      int32_t* leaf_dev = pin;
      // the descriptor stays with the sample (made with it for the default steps) and the tree list with the
      // engine (uploaded when it changes: one forest's calls over many samples upload it once), so the call is
      // one launch and one synchronisation
      const HpState* d_hs = nullptr;
      if (!hp) {
        HpState hs;
        std::memset(&hs, 0, sizeof(hs));
        hs.n_trees = n_trees;
        for (int t = 0; t < n_trees; t++) hs.trees[t] = tree_ids[t];
        if (!e->sample_hs.p || std::memcmp(&hs, &e->sample_hs_host, sizeof(hs)) != 0) {
          e->sample_hs.ensure(sizeof(HpState));
          e->upload_pinned(e->sample_hs.p, &hs, sizeof(hs), w.stream);
          e->sample_hs_host = hs;
        }
        d_hs = e->sample_hs.as<HpState>();
      }
      launch_traverse(hp, grid_desc(e, s, khp, kmp, w.stream), 1, blocks_per_face(fv, hp, g), g,
                      hp ? e->hp_pairs.as<uint4>() : e->mp_pairs.as<uint4>(), hp ? e->hp_tops.as<uint4>() : e->mp_tops.as<uint4>(),
                      hp ? e->hp_topi.as<uint32_t>() : e->mp_topi.as<uint32_t>(), e->trav_top_max,
                      hp ? e->hp_far.as<uint32_t>() : e->mp_far.as<uint32_t>(), d_hs,
                      hp ? e->hp_trees : 0, step, step, f.plane, s->chan.as<uint16_t>(), leaf_dev, e->trav_wg,
                      TRAV_LDS_CAP, w.stream);
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipStreamSynchronize(w.stream));
      for (int i = 0; i < nx; i++)  // rows of the sub-grid: patch (i, j) of the full grid is i * gy + j
        std::memcpy(leaf_ids + (size_t)i * ny * n_trees, pin + (size_t)i * gy * n_trees, (size_t)ny * n_trees * 4);
      return FFD_OK;
    }
  }
  const hipStream_t st = e->main_stream();
  SampleEvalArgs a;
  std::memset(&a, 0, sizeof(a));
  a.nodes = hp ? e->hp_nodes.as<uint4>() : e->mp_nodes.as<uint4>();
  a.roots = hp ? e->hp_roots.as<int32_t>() : e->mp_roots.as<int32_t>();
  a.chan = s->chan.as<uint16_t>();
  a.plane = s->plane;
  a.fint = s->fint;
  a.n_patches = n_patches;
  a.n_trees = n_trees;
  for (int t = 0; t < n_trees; t++) a.trees[t] = tree_ids[t];
  if (grid) {
    a.grid_ny = ny;
    a.x0 = x0;
    a.y0 = y0;
    a.step = step;
  } else if (n_patches <= SAMPLE_INLINE) {
    for (int i = 0; i < 2 * n_patches; i++) a.inl[i] = patches_xy[i];
  } else {
    const size_t b = (size_t)n_patches * 8;
    std::memcpy(e->pin_patch.ensure(b), patches_xy, b);
    e->sample_patches.ensure(b);
    HIP_CHECK(hipMemcpyAsync(e->sample_patches.p, e->pin_patch.p, b, hipMemcpyHostToDevice, st));
    a.patches = e->sample_patches.as<int32_t>();
  }
  const size_t ob = (size_t)n_patches * n_trees * 4;
  a.leaf_out = static_cast<int32_t*>(e->pin_leaf.ensure(ob));  // host-mapped: the kernel writes the results here
  launch_sample_eval(a, st);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipStreamSynchronize(st));
  std::memcpy(leaf_ids, e->pin_leaf.p, ob);
  return FFD_OK;
}

}  // namespace

extern "C" {

ffd_status ffd_sample_create(ffd_engine* e, const uint8_t* gray, int32_t W, int32_t H, int32_t stride, ffd_sample** out) {
  if (e && e->detector_only) return no_forests(e);
  return guarded(e, [&]() -> ffd_status {
    if (!gray || !out || stride < W) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    *out = nullptr;
    if (!sample_size_ok(W, H)) return fail(e, FFD_ERR_UNSUPPORTED, "image sample size unsupported (2..125 wide, 2 rows or more, 255 W H < 2^31)");
    std::unique_ptr<ffd_sample> s(new ffd_sample);
    s->e = e;
    s->device = e->device;
    s->W = W;
    s->H = H;
    s->plane = (int64_t)(H + 1) * PITCH;
    s->chan.ensure((size_t)NCH * s->plane * 2 + 512);  // slack: traversal windows read past a row
    // the face itself is the "image" (copy mode) as in ffd_extract_channels; the channel kernels write
    // straight into the sample's planes
    e->sync_all();
    Workspace& w = *e->ws[0];
    std::vector<uint8_t> bgr((size_t)W * H * 3);
    for (int y = 0; y < H; y++)
      for (int x = 0; x < W; x++) {
        const uint8_t v = gray[(size_t)y * stride + x];  // BGR2GRAY of (v, v, v) is v
        uint8_t* p = &bgr[((size_t)y * W + x) * 3];
        p[0] = p[1] = p[2] = v;
      }
    e->scratch_a.ensure(bgr.size());
    e->upload_pinned(e->scratch_a.p, bgr.data(), bgr.size(), w.stream);
    FaceDesc f;
    std::memset(&f, 0, sizeof(f));
    f.img_w = W; f.img_h = H; f.img_stride = 3 * W; f.bw = W; f.bh = H; f.W = W; f.H = H;
    f.scale = 1.f; f.mode = 0; f.valid = 1;
    f.fint = (int64_t)255 * W * H >= (int64_t)1 << 24 ? 1 : 0;  // OpenCV's float integral rounds past 2^24
    s->fint = f.fint;
    f.plane = s->plane;
    w.gray.ensure((size_t)H * PITCH + 256);
    w.mag.ensure((size_t)NGABOR * H * PITCH * 4 + 256);
    w.gabor_redo.ensure(5 * 4);
    if (w.gabor_mm.n < 5 * 64) {
      w.gabor_mm.ensure(5 * 64);
      HIP_CHECK(hipMemsetAsync(w.gabor_mm.p, 0, w.gabor_mm.n, w.stream));
    }
    e->upload_descriptors(w.faces, std::vector<FaceDesc>{f}, w.stream);
    const FaceDesc* dfd = w.faces.as<FaceDesc>();
    launch_gray_resize(dfd, 1, e->scratch_a.as<uint8_t>(), w.gray.as<uint8_t>(), w.stream);
    // the five Gabor scales and the integrals side by side on the workspace's fork streams, as a small batch
    // runs them (run_chunk): one face's kernels are each a few workgroups, so in one stream they would run
    // one after another (≈ 0.33 ms of a sample's ≈ 0.45 ms, evaluate_mt trace)
    const int nfork = (int)w.fork.size();
    HIP_CHECK(hipEventRecord(w.fork_ev[0], w.stream));
    for (int i = 0; i < nfork; i++) HIP_CHECK(hipStreamWaitEvent(w.fork[i], w.fork_ev[0], 0));
    auto cs = [&](int i) { return i % (nfork + 1) == 0 ? w.stream : w.fork[i % (nfork + 1) - 1]; };
    for (int nu = 4; nu >= 0; nu--)
      launch_gabor(nu, dfd, 1, H, w.gray.as<uint8_t>(), e->gabor_coef.as<float>(), w.mag.as<float>(),
                   s->chan.as<uint16_t>(), w.gabor_redo.as<int>(), e->gabor_exact, w.gabor_mm.as<uint32_t>(), cs(4 - nu));
    launch_integral(dfd, 1, H, w.gray.as<uint8_t>(), s->chan.as<uint16_t>(), cs(5));
    HIP_CHECK(hipGetLastError());
    for (int i = 0; i < nfork; i++) {
      HIP_CHECK(hipEventRecord(w.fork_ev[1 + i], w.fork[i]));
      HIP_CHECK(hipStreamWaitEvent(w.stream, w.fork_ev[1 + i], 0));
    }
    grid_desc(e, s.get(), e->desc.hp_option.step_size, e->desc.mp_option.step_size, w.stream);
    HIP_CHECK(hipStreamSynchronize(w.stream));  // bgr is released on return
    w.count = 0;
    w.pending = false;
    if (e->last_ws == 0) e->last_ws = -1;
    *out = s.release();
    e->track_sample(*out);
    return FFD_OK;
  });
}

ffd_status ffd_sample_create_from_channels(ffd_engine* e, const uint32_t* channels, int32_t W, int32_t H,
                                           ffd_sample** out) {
  if (e && e->detector_only) return no_forests(e);
  return guarded(e, [&]() -> ffd_status {
    if (!channels || !out) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    *out = nullptr;
    if (!sample_size_ok(W, H)) return fail(e, FFD_ERR_UNSUPPORTED, "image sample size unsupported (2..125 wide, 2 rows or more, 255 W H < 2^31)");
    std::unique_ptr<ffd_sample> s(new ffd_sample);
    s->e = e;
    s->device = e->device;
    s->W = W;
    s->H = H;
    s->plane = (int64_t)(H + 1) * PITCH;
    std::vector<uint16_t> J((size_t)NCH * s->plane, 0);
    uint32_t vmax = 0;
    for (int c = 0; c < NCH; c++)
      for (int y = 0; y <= H; y++)
        for (int x = 0; x <= W; x++) {
          const uint32_t v = channels[((size_t)c * (H + 1) + y) * (W + 1) + x];
          vmax = std::max(vmax, v);
          J[(size_t)c * s->plane + (size_t)y * PITCH + x] = (uint16_t)v;
        }
    if (vmax >= FINT_LIMIT) return fail(e, FFD_ERR_UNSUPPORTED, "integral values of 2^31 or more (rect_mean_fint window)");
    s->fint = vmax >= (1u << 24) ? 1 : 0;  // float-rounded integrals (CV_32F past 2^24)
    s->chan.ensure(J.size() * 2 + 512);
    HIP_CHECK(hipMemcpyAsync(s->chan.p, J.data(), J.size() * 2, hipMemcpyHostToDevice, e->main_stream()));
    grid_desc(e, s.get(), e->desc.hp_option.step_size, e->desc.mp_option.step_size, e->main_stream());
    HIP_CHECK(hipStreamSynchronize(e->main_stream()));
    *out = s.release();
    e->track_sample(*out);
    return FFD_OK;
  });
}

void ffd_sample_destroy(ffd_sample* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  if (s->e) {
    s->e->untrack_sample(s);
    (void)hipStreamSynchronize(s->e->main_stream());
  }
  delete s;  // (an orphaned sample's planes were freed with its engine)
}

ffd_status ffd_sample_size(const ffd_sample* s, int32_t* W, int32_t* H) {
  if (!s) return FFD_ERR_INVALID_ARGUMENT;  // (valid on an orphaned sample too)
  if (W) *W = s->W;
  if (H) *H = s->H;
  return FFD_OK;
}

ffd_status ffd_sample_channels(const ffd_sample* s, uint32_t* out) {
  if (!s) return FFD_ERR_INVALID_ARGUMENT;
  if (!s->e) return orphaned();
  return guarded(s->e, [&]() -> ffd_status {
    if (!out) return fail(s->e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    std::vector<uint16_t> v((size_t)NCH * s->plane);
    HIP_CHECK(hipMemcpyAsync(v.data(), s->chan.p, v.size() * 2, hipMemcpyDeviceToHost, s->e->main_stream()));
    HIP_CHECK(hipStreamSynchronize(s->e->main_stream()));
    widen_integrals(v.data(), s->plane, s->W, s->H, out);
    return FFD_OK;
  });
}

ffd_status ffd_sample_eval_leaves(ffd_sample* s, int32_t kind, const int32_t* patches_xy, int32_t n_patches,
                                  const int32_t* tree_ids, int32_t n_trees, int32_t* leaf_ids) {
  if (!s) return FFD_ERR_INVALID_ARGUMENT;
  if (!s->e) return orphaned();
  return guarded(s->e, [&]() -> ffd_status {
    if (!patches_xy && n_patches) return fail(s->e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    static const int32_t none[2] = {0, 0};
    return sample_eval(s, kind, patches_xy ? patches_xy : none, n_patches, 0, 0, 0, 0, 0, tree_ids, n_trees, leaf_ids);
  });
}

ffd_status ffd_sample_eval_grid(ffd_sample* s, int32_t kind, int32_t x0, int32_t y0, int32_t step, int32_t nx,
                                int32_t ny, const int32_t* tree_ids, int32_t n_trees, int32_t* leaf_ids) {
  if (!s) return FFD_ERR_INVALID_ARGUMENT;
  if (!s->e) return orphaned();
  return guarded(s->e, [&]() -> ffd_status {
    return sample_eval(s, kind, nullptr, 0, x0, y0, step, nx, ny, tree_ids, n_trees, leaf_ids);
  });
}

ffd_status ffd_sample_estimate_headpose(ffd_sample* s, const ffd_rect* region, const ffd_headpose_option* options,
                                        float* headpose, float* variance) {
  if (!s) return FFD_ERR_INVALID_ARGUMENT;
  if (!s->e) return orphaned();
  ffd_engine* e = s->e;
  return guarded(e, [&]() -> ffd_status {
    const ffd_rect full{0, 0, s->W, s->H};
    if (!region) region = &full;
    if (!region_ok(s->W, s->H, region)) return fail(e, FFD_ERR_INVALID_ARGUMENT, "face_bbox outside the image sample");
    const ffd_headpose_option o = options ? *options : e->desc.hp_option;
    if (o.step_size <= 0) return fail(e, FFD_ERR_INVALID_ARGUMENT, "invalid HeadPoseEstimatorOption");
    e->sync_all();
    Workspace& w = *e->ws[0];
    HpState hs;
    if (region->x == 0 && region->y == 0 && region->width == s->W && region->height == s->H) {
      const FaceDesc f = sample_desc(s, o.step_size, e->desc.mp_option.step_size, e->mp_step_y());
      stage_desc(e, w, f);
      hs = run_headpose(e, w, f, s->chan.as<uint16_t>(), o);
    } else {  // a sub-region: its integrals relative to the region origin (stage_sample)
      std::vector<uint32_t> ch((size_t)NCH * (s->H + 1) * (s->W + 1));
      const ffd_status st = ffd_sample_channels(s, ch.data());
      if (st != FFD_OK) return st;
      const FaceDesc f = stage_sample(e, w, ch.data(), s->W, s->H, *region, o.step_size, e->desc.mp_option.step_size,
                                      e->mp_step_y());
      hs = run_headpose(e, w, f, w.chan.as<uint16_t>(), o);
    }
    if (headpose) *headpose = hs.headpose;
    if (variance) *variance = hs.variance;
    return FFD_OK;
  });
}

ffd_status ffd_sample_estimate_facial_features(ffd_sample* s, const ffd_rect* region, const int32_t* tree_ids,
                                               int32_t n_trees, const ffd_multipart_option* options, int32_t* points) {
  if (!s) return FFD_ERR_INVALID_ARGUMENT;
  if (!s->e) return orphaned();
  ffd_engine* e = s->e;
  return guarded(e, [&]() -> ffd_status {
    if (!points) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    const ffd_rect full{0, 0, s->W, s->H};
    if (!region) region = &full;
    if (!region_ok(s->W, s->H, region)) return fail(e, FFD_ERR_INVALID_ARGUMENT, "face_bbox outside the image sample");
    const ffd_multipart_option o = options ? *options : e->desc.mp_option;
    const ffd_status cst = check_mp_call(e, tree_ids, n_trees, o);
    if (cst != FFD_OK) return cst;
    const int step_y = o.step_size_y > 0 ? o.step_size_y : o.step_size;
    e->sync_all();
    Workspace& w = *e->ws[0];
    if (region->x == 0 && region->y == 0 && region->width == s->W && region->height == s->H) {
      const FaceDesc f = sample_desc(s, e->desc.hp_option.step_size, o.step_size, step_y);
      stage_desc(e, w, f);
      run_facial_features(e, w, f, s->chan.as<uint16_t>(), tree_ids, n_trees, o, points);
    } else {
      std::vector<uint32_t> ch((size_t)NCH * (s->H + 1) * (s->W + 1));
      const ffd_status st = ffd_sample_channels(s, ch.data());
      if (st != FFD_OK) return st;
      const FaceDesc f = stage_sample(e, w, ch.data(), s->W, s->H, *region, e->desc.hp_option.step_size, o.step_size,
                                      step_y);
      run_facial_features(e, w, f, w.chan.as<uint16_t>(), tree_ids, n_trees, o, points);
    }
    return FFD_OK;
  });
}

// MeanShift::shift (MeanShift.hpp:41-76) of one vote list: the list as landmark 0 of a one-face chunk
// (tslots 1, nmx = the list length) through the engine's MeanShift kernel.
ffd_status ffd_meanshift(ffd_engine* e, const ffd_vote* votes, int32_t n, const ffd_meanshift_option* option,
                         float* mean_xy) {
  return guarded(e, [&]() -> ffd_status {
    if ((n && !votes) || n < 0 || !mean_xy) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    const ffd_meanshift_option o = option ? *option : e->desc.ms_option;
    if (o.max_iterations < 0 || o.kernel_size <= 0) return fail(e, FFD_ERR_INVALID_ARGUMENT, "invalid MeanShiftOption");
    // positions beyond int16 (or FFD_VOTES_WIDE): the list as VoteW records (a wide face)
    bool wide = e->force_wide;
    for (int i = 0; i < n && !wide; i++)
      wide = votes[i].check && (votes[i].x < -32768 || votes[i].x > 32767 || votes[i].y < -32768 || votes[i].y > 32767);
    std::vector<VoteW> v;  // (narrow: packed as Vote below)
    v.reserve(n);
    for (int i = 0; i < n; i++) {
      if (!votes[i].check) continue;  // getMean / getWeightedMean skip unchecked votes
      v.push_back(VoteW{votes[i].x, votes[i].y, votes[i].weight, 0});
    }
    e->sync_all();
    Workspace& w = *e->ws[0];
    FaceDesc f;
    std::memset(&f, 0, sizeof(f));
    f.valid = 1; f.nochan = 1; f.scale = 1.f; f.wide = wide;
    f.nmx = std::max<int>(1, (int)v.size());
    f.nmy = 1;
    int32_t counts[NPARTS] = {(int32_t)v.size()};
    w.votes.ensure(std::max<size_t>(1, v.size()) * sizeof(VoteW));
    if (wide) {
      if (!v.empty()) HIP_CHECK(hipMemcpyAsync(w.votes.p, v.data(), v.size() * sizeof(VoteW), hipMemcpyHostToDevice, w.stream));
    } else {
      std::vector<Vote> p(v.size());
      for (size_t i = 0; i < v.size(); i++) p[i] = Vote{(int16_t)v[i].x, (int16_t)v[i].y, v[i].w};
      if (!p.empty()) HIP_CHECK(hipMemcpyAsync(w.votes.p, p.data(), p.size() * sizeof(Vote), hipMemcpyHostToDevice, w.stream));
      HIP_CHECK(hipStreamSynchronize(w.stream));  // p is released on return
    }
    w.vote_counts.ensure(sizeof(counts));
    HIP_CHECK(hipMemcpyAsync(w.vote_counts.p, counts, sizeof(counts), hipMemcpyHostToDevice, w.stream));
    w.ms_mean.ensure(NPARTS * 2 * 4);
    e->out.ensure(sizeof(FaceOut));
    std::vector<FaceDesc> one{f};
    upload(w.faces, one, w.stream);
    launch_meanshift(w.faces.as<FaceDesc>(), 1, nullptr, 1, 1, (float)o.kernel_size, o.max_iterations,
                     o.stopping_criteria, w.votes.as<Vote>(), w.vote_counts.as<int32_t>(), w.ms_mean.as<float>(),
                     e->out.as<FaceOut>(), nullptr, w.stream, wide);
    HIP_CHECK(hipGetLastError());
    float m[2];
    HIP_CHECK(hipMemcpyAsync(m, w.ms_mean.p, sizeof(m), hipMemcpyDeviceToHost, w.stream));
    HIP_CHECK(hipStreamSynchronize(w.stream));
    w.count = 0;
    w.pending = false;
    if (e->last_ws == 0) e->last_ws = -1;
    mean_xy[0] = m[0];
    mean_xy[1] = m[1];
    return FFD_OK;
  });
}

}  // extern "C"
