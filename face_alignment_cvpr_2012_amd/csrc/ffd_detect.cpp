// ffd_detect.cpp — host side of the Haar face detector and the frame-level
// entry points built on it:
//   ffd_detect_faces[_device]  FaceForest::detectFace      /root/reference/src/FaceForest.cpp:136-159
//   ffd_analyze_images         FaceForest::analyzeImage    /root/reference/src/FaceForest.cpp:161-181
//   ffd_detect_candidates      (test hook) detectMultiScale's ungrouped candidates of one frame
// The pyramid geometry (which scales detectMultiScale scans, their sizes and resize modes) is built
// here with the restatement's double arithmetic (oracle/ffd_oracle.cpp haar_scan); all pixel work runs
// in the ffd_haar.hip kernels on the engine's main stream.
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ffd_engine_impl.hpp"
#include "model_io.hpp"

using namespace ffd_host;

// Load the cascade arrays written by ffd_convert (haar.*) into device records.
void ffd_engine::load_cascade(const ffd::ModelFile& m) {
  have_haar = m.has("haar.window");
  if (!have_haar) return;
  const int32_t* win = m.get("haar.window").as<int32_t>();
  haar_ww = win[0];
  haar_wh = win[1];
  if (haar_ww < 3 || haar_wh < 3 || haar_ww > 255 || haar_wh > 255) throw std::runtime_error("cascade window size");
  // the squared integral is kept modulo 2^32: exact for the normrect's sum while (ww - 2)(wh - 2) 255^2 < 2^32
  if ((int64_t)(haar_ww - 2) * (haar_wh - 2) * 255 * 255 >= ((int64_t)1 << 32)) throw std::runtime_error("cascade window too large");
  const auto& sf = m.get("haar.stage_first");
  const auto& sn = m.get("haar.stage_ntrees");
  const auto& st = m.get("haar.stage_threshold");
  haar_stages = (int)sf.count();
  std::vector<HaarStage> stages(haar_stages);
  for (int s = 0; s < haar_stages; s++) {
    stages[s].first = sf.as<int32_t>()[s];
    stages[s].ntrees = sn.as<int32_t>()[s];
    stages[s].thr = st.as<float>()[s] - 1e-5f;  // CascadeClassifier::Data::read THRESHOLD_EPS
    stages[s].n_two = 0;
    stages[s].n_sh = 0;
  }
  const auto& wf = m.get("haar.weak_feature");
  const auto& wt = m.get("haar.weak_threshold");
  const auto& wl = m.get("haar.weak_leaves");
  const auto& fr = m.get("haar.feature_rect");
  const auto& fw = m.get("haar.feature_weight");
  const int64_t nw = (int64_t)wf.count(), nf = (int64_t)fw.count() / 3;
  // one table per ystep (1: factor > 2, 2 otherwise; detectMultiScale's yStep): the corner offsets
  // depend on the LDS window's row pitch
  std::vector<HaarWeak> weak(2 * nw);
  for (int ys = 1; ys <= 2; ys++) {
    const int WC = haar_window_cols(ys, haar_ww);
    for (int64_t i = 0; i < nw; i++) {
      const int f = wf.as<int32_t>()[i];
      if (f < 0 || f >= nf) throw std::runtime_error("cascade feature index out of range");
      const int32_t* r = fr.as<int32_t>() + f * 12;
      HaarWeak& w = weak[(ys - 1) * nw + i];
      std::memset(&w, 0, sizeof(w));
      w.w0 = fw.as<float>()[f * 3];
      w.w1 = fw.as<float>()[f * 3 + 1];
      w.w2 = fw.as<float>()[f * 3 + 2];
      for (int k = 0; k < 3; k++) {
        if (k == 2 && w.w2 == 0.0f) break;  // two-rectangle feature: rect 2 stays empty (offsets 0)
        for (int j = 0; j < 4; j++)
          if (r[4 * k + j] < 0 || r[4 * k + j] > 255) throw std::runtime_error("cascade rectangle out of range");
        if (r[4 * k] + r[4 * k + 2] > haar_ww || r[4 * k + 1] + r[4 * k + 3] > haar_wh)
          throw std::runtime_error("cascade rectangle outside the window");
        const int x = r[4 * k], y = r[4 * k + 1], rw = r[4 * k + 2], rh = r[4 * k + 3];
        const uint32_t a = (uint32_t)haar_window_offset(ys, WC, y, x), b = (uint32_t)haar_window_offset(ys, WC, y, x + rw);
        const uint32_t c = (uint32_t)haar_window_offset(ys, WC, y + rh, x);
        const uint32_t d = (uint32_t)haar_window_offset(ys, WC, y + rh, x + rw);
        if (d > 0xFFFFu || b > 0xFFFFu) throw std::runtime_error("cascade window too large");
        w.o[2 * k] = a | b << 16;
        w.o[2 * k + 1] = c | d << 16;
      }
      w.thr = wt.as<float>()[i];
      w.leaf0 = wl.as<float>()[2 * i];
      w.leaf1 = wl.as<float>()[2 * i + 1];
    }
  }
  haar_nweak = (int)nw;
  for (const auto& s : stages)
    if (s.first < 0 || s.ntrees < 0 || s.first + s.ntrees > nw) throw std::runtime_error("cascade stage range");
  // Two-rectangle classifiers first within each stage (HaarStage::n_two of them), so the kernel reads
  // 8 window corners for those instead of 12.  This reorders predictOrderedStump's double sum of the
  // stage's float leaves, which is exact in any order when every partial sum is representable:
  // all leaves are integer multiples of 2^e (e = the smallest leaf's last mantissa bit) and the sum of
  // the largest |leaf| per classifier stays below 2^(53 + e).  A stage that fails the check keeps its
  // order (n_two = 0: every classifier through the 12-corner form, which covers rect 2 empty).
  // Two rectangles sharing two corners (an edge segment; they then have opposite signs in both rectangles' sums
  // tl - tr - bl + br): rewritten as HAAR_SHARED records (ffd_haar.hpp).  Corners are LDS offsets, equal offsets
  // being the same window corner.
  struct Corner {
    uint32_t off;
    int sign;
  };
  auto corners = [](const HaarWeak& w, int k, Corner* c) {
    c[0] = {w.o[2 * k] & 0xFFFFu, +1};
    c[1] = {w.o[2 * k] >> 16, -1};
    c[2] = {w.o[2 * k + 1] & 0xFFFFu, -1};
    c[3] = {w.o[2 * k + 1] >> 16, +1};
  };
  auto shared_of = [&](const HaarWeak& w, Corner* s1, Corner* s2) {  // the two shared corners, s1 added by rect 0
    Corner a[4], b[4];
    corners(w, 0, a);
    corners(w, 1, b);
    for (int i = 0; i < 4; i++)
      for (int j = i + 1; j < 4; j++)
        if (a[i].off == a[j].off || b[i].off == b[j].off) return false;  // (a degenerate rectangle)
    int n = 0;
    Corner sc[4];
    for (const Corner& x : a)
      for (const Corner& y : b)
        if (x.off == y.off) sc[n++] = x;
    if (n != 2 || sc[0].sign == sc[1].sign) return false;
    *s1 = sc[0].sign > 0 ? sc[0] : sc[1];
    *s2 = sc[0].sign > 0 ? sc[1] : sc[0];
    return true;
  };
  auto shared_corners = [&](int64_t i) {  // both ystep tables share the pattern (same rectangles)
    Corner s1, s2;
    return shared_of(weak[i], &s1, &s2) && shared_of(weak[nw + i], &s1, &s2);
  };
  auto to_shared = [&](const HaarWeak& w) {
    Corner s1, s2, a[4], b[4];
    shared_of(w, &s1, &s2);
    corners(w, 0, a);
    corners(w, 1, b);
    HaarWeak r = w;
    r.o[0] = s1.off | s2.off << 16;
    uint32_t x1 = 0, x2 = 0, y1 = 0, y2 = 0;
    for (const Corner& c : a)  // rect 0 = S1 - S2 - X1 + X2
      if (c.off != s1.off && c.off != s2.off) (c.sign > 0 ? x2 : x1) = c.off;
    int sign1 = 0;  // rect 1 adds S1 (+1) or subtracts it (-1): rect 1 = sign1 (E - Y1 + Y2)
    for (const Corner& c : b)
      if (c.off == s1.off) sign1 = c.sign;
    for (const Corner& c : b)
      if (c.off != s1.off && c.off != s2.off) (c.sign * sign1 > 0 ? y2 : y1) = c.off;
    r.o[1] = x1 | x2 << 16;
    r.o[2] = y1 | y2 << 16;
    r.o[3] = HAAR_SHARED;
    r.o[4] = r.o[5] = 0;
    r.w1 = sign1 > 0 ? w.w1 : -w.w1;  // w1 * (float)(-t) == (-w1) * (float)t exactly
    return r;
  };
  haar_order_free = 1;
  for (auto& st : stages) {
    int emin = INT32_MAX;
    double bound = 0.0;
    for (int i = st.first; i < st.first + st.ntrees; i++) {
      const HaarWeak& w = weak[i];
      for (float l : {w.leaf0, w.leaf1})
        if (l != 0.0f) {
          int ex;
          std::frexp((double)l, &ex);
          emin = std::min(emin, ex - 24);
        }
      bound += std::max(std::fabs((double)w.leaf0), std::fabs((double)w.leaf1));
    }
    st.n_two = 0;
    st.n_sh = 0;
    if (st.ntrees == 0 || emin == INT32_MAX) continue;  // a sum of zeros: exact in any order
    if (!(bound < std::ldexp(1.0, 52 + emin))) {
      haar_order_free = 0;
      continue;
    }
    // the shared-corner two-rectangle classifiers first, then the other two-rectangle ones, then the rest
    std::vector<int> sh, two, three;
    for (int i = st.first; i < st.first + st.ntrees; i++)
      (weak[i].w2 != 0.0f ? three : shared_corners(i) ? sh : two).push_back(i);
    std::vector<HaarWeak> perm;
    for (int t = 0; t < 2; t++) {
      perm.clear();
      for (int i : sh) perm.push_back(to_shared(weak[t * nw + i]));
      for (int i : two) perm.push_back(weak[t * nw + i]);
      for (int i : three) perm.push_back(weak[t * nw + i]);
      std::copy(perm.begin(), perm.end(), weak.begin() + t * nw + st.first);
    }
    st.n_sh = (int)sh.size();
    st.n_two = (int)(sh.size() + two.size());
  }
  upload(haar_weak, weak, main_stream());
  upload(haar_stage, stages, main_stream());
}

namespace {

struct FrameIn {
  int64_t img_off;
  int w, h, stride;
};

void default_options(ffd_detect_options* o) {
  o->min_feature_size = 30;     // FaceDetectionOption (include/FaceForest.hpp:21-32)
  o->min_neighbors = 1;
  o->search_scale_factor = 1.3f;
  o->widen = 1;
}

// detectMultiScale's pyramid (oracle haar_scan) for every frame -> levels; returns false if a frame
// is smaller than the cascade window at every scale (no levels)
void build_levels(const ffd_engine* e, const std::vector<FrameIn>& in, const ffd_detect_options& o,
                  std::vector<HaarFrame>& frames, std::vector<HaarLevel>& levels, int64_t sizes[4]) {
  frames.clear();
  levels.clear();
  int64_t gray = 0, scaled = 0, sums = 0, res = 0;
  const double sf = (double)o.search_scale_factor;
  for (size_t k = 0; k < in.size(); k++) {
    HaarFrame f;
    std::memset(&f, 0, sizeof(f));
    f.img_off = in[k].img_off;
    f.gray_off = gray;
    f.w = in[k].w;
    f.h = in[k].h;
    f.stride = in[k].stride;
    f.level0 = (int)levels.size();
    gray += align_up((int64_t)f.w * f.h, 256);
    int rows = 0;
    for (double factor = 1;; factor *= sf) {
      const int winW = (int)std::nearbyint(e->haar_ww * factor), winH = (int)std::nearbyint(e->haar_wh * factor);
      const int sW = (int)std::nearbyint(f.w / factor), sH = (int)std::nearbyint(f.h / factor);
      const int pW = sW - e->haar_ww, pH = sH - e->haar_wh;
      if (pW <= 0 || pH <= 0) break;
      if (winW > f.w || winH > f.h) break;  // maxObjectSize = image size
      if (winW < o.min_feature_size || winH < o.min_feature_size) continue;
      HaarLevel L;
      std::memset(&L, 0, sizeof(L));
      L.gray_off = f.gray_off;
      L.img_off = scaled;
      L.sum_off = sums;
      L.res_off = res;
      L.factor = factor;
      L.src_w = f.w;
      L.src_h = f.h;
      L.sw = sW;
      L.sh = sH;
      L.ystep = factor > 2. ? 1 : 2;
      L.nx = (pW + L.ystep - 1) / L.ystep;
      L.ny = (pH + L.ystep - 1) / L.ystep;
      L.win_w = winW;
      L.win_h = winH;
      if (sW == f.w && sH == f.h) {
        L.mode = 0;
      } else {  // resize()'s INTER_LINEAR -> INTER_AREA 2x switch (oracle cv_resize)
        L.scale_x = 1. / ((double)sW / f.w);
        L.scale_y = 1. / ((double)sH / f.h);
        const int ix = (int)std::nearbyint(L.scale_x), iy = (int)std::nearbyint(L.scale_y);
        const bool area_fast = std::fabs(L.scale_x - ix) < DBL_EPSILON && std::fabs(L.scale_y - iy) < DBL_EPSILON;
        L.mode = (area_fast && ix == 2 && iy == 2) ? 2 : 1;
      }
      int xv = 0;
      while (xv <= sW - 16) xv += 16;
      while (xv < sW - 4) xv += 4;
      L.xv = xv;
      L.row0 = rows;
      L.frame = (int)k;
      rows += L.ny;
      scaled += align_up((int64_t)sW * sH, 256);
      sums += align_up((int64_t)(sW + 1) * (sH + 1), 64);
      res += align_up((int64_t)L.nx * L.ny, 256);
      levels.push_back(L);
    }
    f.level1 = (int)levels.size();
    f.rows = rows;
    frames.push_back(f);
  }
  sizes[0] = gray;
  sizes[1] = scaled;
  sizes[2] = sums;
  sizes[3] = res;
}

// Run the detector over frames already in device memory (e->main_stream()); boxes per frame out.
// Frames go through in groups (FFD_DETECT_GROUP frames, default 64) so the pyramid / integral /
// survivor buffers stay bounded whatever the batch.
// cap: raw candidates per frame the collection and grouping hold; a frame with more is run again on its own
// with a capacity that holds all of them (detectMultiScale has no limit, FaceForest.cpp:146).
ffd_status detect_batch(ffd_engine* e, const uint8_t* d_images, const std::vector<FrameIn>& all_in,
                        const ffd_detect_options& o, std::vector<std::vector<ffd_rect>>& out,
                        std::vector<std::vector<ffd_rect>>* raw, int cap = 0) {
  if (!e->have_haar) return fail(e, FFD_ERR_MODEL, "the model has no Haar cascade (convert it with ffd_convert)");
  if (!(o.search_scale_factor > 1.f) || o.min_feature_size < 0)
    return fail(e, FFD_ERR_INVALID_ARGUMENT, "search_scale_factor must be > 1 and min_feature_size >= 0");
  for (const auto& f : all_in)
    if (f.w > 32767 || f.h > 32767) return fail(e, FFD_ERR_UNSUPPORTED, "frames wider or taller than 32767 pixels");
  out.assign(all_in.size(), {});
  if (raw) raw->assign(all_in.size(), {});
  int group = 64;
  if (const char* v = std::getenv("FFD_DETECT_GROUP")) group = std::max(1, std::atoi(v));
  hipStream_t s = e->main_stream();
  // (FFD_DETECT_CAP / FFD_DETECT_RERUN_CAP: test hooks that force the overflow re-runs with small frames)
  const int rerun_min = std::getenv("FFD_DETECT_RERUN_CAP") ? std::atoi(std::getenv("FFD_DETECT_RERUN_CAP")) : 0;
  if (cap <= 0) cap = std::getenv("FFD_DETECT_CAP") ? std::max(16, std::atoi(std::getenv("FFD_DETECT_CAP"))) : HAAR_MAX_CAND;
  if (cap > HAAR_MAX_CAND) group = 1;
  for (size_t g0 = 0; g0 < all_in.size(); g0 += group) {
    const std::vector<FrameIn> in(all_in.begin() + g0, all_in.begin() + std::min(all_in.size(), g0 + group));
    std::vector<HaarFrame> frames;
    std::vector<HaarLevel> levels;
    int64_t sz[4];
    build_levels(e, in, o, frames, levels, sz);
    const int nF = (int)frames.size(), nL = (int)levels.size();
    upload(e->det_frames, frames, s);
    e->det_gray.ensure(sz[0]);
    e->det_ncand.ensure((size_t)nF * 8);
    e->det_cand.ensure((size_t)nF * cap * 16);
    e->det_clsrect.ensure((size_t)nF * cap * 16);
    e->det_clssum.ensure((size_t)nF * cap * 20);
    e->det_boxes.ensure((size_t)nF * cap * 16);
    e->det_packed.ensure((size_t)nF * cap * 20);
    if (cap > HAAR_MAX_CAND) e->det_label.ensure(((size_t)nF * cap + 1) * 4);  // (+ the rounds' change flag)
    int max_px = 0, max_lpx = 0, max_rows = 0, max_cols = 0, max_ystep = 1;
    for (const auto& f : frames) max_px = std::max(max_px, f.w * f.h);
    int total_tiles = 0;  // the cascade's grid: every level's tiles, none empty (HaarLevel::tile0)
    for (auto& L : levels) {
      L.tile0 = total_tiles;
      total_tiles += ((L.nx + HAAR_TILE_X - 1) / HAAR_TILE_X) * ((L.ny + HAAR_TILE_Y - 1) / HAAR_TILE_Y);
      max_lpx = std::max(max_lpx, L.sw * L.sh);
      max_rows = std::max(max_rows, L.sh);
      max_cols = std::max(max_cols, L.sw);
      max_ystep = std::max(max_ystep, L.ystep);
    }
    int32_t* n_cand = e->det_ncand.as<int32_t>();
    int32_t* n_boxes = n_cand + nF;
    if (nL > 0) {
      upload(e->det_levels, levels, s);
      e->det_scaled.ensure(sz[1]);
      e->det_sum.ensure(sz[2] * 4);
      e->det_sq.ensure(sz[2] * 4);
      e->det_res.ensure(sz[3]);
      launch_haar_gray(e->det_frames.as<HaarFrame>(), nF, max_px, d_images, e->det_gray.as<uint8_t>(), s);
      launch_haar_pyramid(e->det_levels.as<HaarLevel>(), nL, max_lpx, max_rows, max_cols, e->det_gray.as<uint8_t>(),
                          e->det_scaled.as<uint8_t>(), e->det_sum.as<int32_t>(), e->det_sq.as<uint32_t>(), s);
      const int lds = haar_cascade_lds(max_ystep, e->haar_ww, e->haar_wh);
      if (lds > 64 * 1024) return fail(e, FFD_ERR_UNSUPPORTED, "cascade window too large for the LDS tile");
      launch_haar_cascade(e->det_levels.as<HaarLevel>(), nL, total_tiles, e->det_sum.as<int32_t>(),
                          e->det_sq.as<uint32_t>(), e->haar_weak.as<HaarWeak>(), e->haar_nweak, e->haar_stage.as<HaarStage>(),
                          e->haar_stages, e->haar_ww, e->haar_wh, e->haar_order_free, e->det_res.as<int8_t>(), lds, s);
    }
    int max_frame_rows = 0;
    for (const auto& f : frames) max_frame_rows = std::max(max_frame_rows, f.rows);
    e->det_rowcnt.ensure((size_t)nF * std::max(1, max_frame_rows) * 4);
    const int grc = launch_haar_group(e->det_frames.as<HaarFrame>(), nF, max_frame_rows, e->det_rowcnt.as<int32_t>(), nL > 0 ? e->det_levels.as<HaarLevel>() : nullptr,
                      nL > 0 ? e->det_res.as<int8_t>() : nullptr, cap, e->det_cand.as<int4>(), n_cand,
                      o.min_neighbors, o.widen, e->det_clsrect.as<int4>(), e->det_clssum.as<int>(),
                      e->det_boxes.as<int4>(), n_boxes, cap > HAAR_MAX_CAND ? e->det_label.as<int>() : nullptr, s);
    if (grc == HAAR_GROUP_HIP_ERROR) throw HipError("detector grouping: a HIP call of the label rounds failed");
    if (grc == HAAR_GROUP_NO_CONVERGENCE) throw std::runtime_error("detector grouping: label rounds did not converge");
    int4* packed = e->det_packed.as<int4>();
    int32_t* owner = reinterpret_cast<int32_t*>(packed + (size_t)nF * cap);
    launch_haar_pack(nF, cap, e->det_boxes.as<int4>(), n_boxes, packed, owner, s);
    std::vector<int32_t> counts(2 * nF);
    HIP_CHECK(hipMemcpyAsync(counts.data(), n_cand, 2 * nF * 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    int64_t total = 0;  // packed boxes of the group, every frame's
    std::vector<char> over(nF, 0);  // frames whose raw candidates exceed cap: boxes from a run of their own
    for (int k = 0; k < nF; k++) {
      if (counts[k] > cap) {
        if (counts[k] > HAAR_GROUP_MAX)  // (the pair tests grow as N^2, ffd_haar.hpp)
          return fail(e, FFD_ERR_UNSUPPORTED, "frame " + std::to_string(g0 + k) + ": " + std::to_string(counts[k]) +
                                                  " raw detections (more than " + std::to_string(HAAR_GROUP_MAX) + ")");
        over[k] = 1;
      }
      total += counts[nF + k];
    }
    std::vector<int4> pb(total);
    std::vector<int32_t> po(total);
    if (total > 0) {
      HIP_CHECK(hipMemcpyAsync(pb.data(), packed, total * sizeof(int4), hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipMemcpyAsync(po.data(), owner, total * sizeof(int32_t), hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipStreamSynchronize(s));
    }
    for (int64_t i = 0; i < total; i++)
      if (!over[po[i]]) out[g0 + po[i]].push_back(ffd_rect{pb[i].x, pb[i].y, pb[i].z, pb[i].w});
    if (raw) {
      for (int k = 0; k < nF; k++) {
        if (over[k]) continue;
        std::vector<int4> tmp(counts[k]);
        if (counts[k] > 0) {
          HIP_CHECK(hipMemcpyAsync(tmp.data(), e->det_cand.as<int4>() + (int64_t)k * cap, counts[k] * sizeof(int4),
                                   hipMemcpyDeviceToHost, s));
          HIP_CHECK(hipStreamSynchronize(s));
        }
        for (const int4& b : tmp) (*raw)[g0 + k].push_back(ffd_rect{b.x, b.y, b.z, b.w});
      }
    }
    for (int k = 0; k < nF; k++) {
      if (!over[k]) continue;
      std::vector<std::vector<ffd_rect>> o1, r1;
      const int cap1 = std::max(rerun_min, (counts[k] + 1023) / 1024 * 1024);
      const ffd_status st = detect_batch(e, d_images, {in[k]}, o, o1, raw ? &r1 : nullptr, cap1);
      if (st != FFD_OK) return st;
      out[g0 + k] = o1[0];
      if (raw) (*raw)[g0 + k] = r1[0];
    }
  }
  return FFD_OK;
}

// upload host frames into the engine's image staging buffer
ffd_status upload_frames(ffd_engine* e, const ffd_image* imgs, int32_t n_img, std::vector<FrameIn>& in) {
  if (n_img < 0 || (n_img > 0 && !imgs)) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad image list");
  in.resize(n_img);
  int64_t total = 0;
  for (int i = 0; i < n_img; i++) {
    if (!imgs[i].bgr || imgs[i].width <= 0 || imgs[i].height <= 0 || imgs[i].stride < 3 * imgs[i].width)
      return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad image " + std::to_string(i));
    in[i] = FrameIn{total, imgs[i].width, imgs[i].height, imgs[i].stride};
    total += align_up((int64_t)imgs[i].stride * imgs[i].height, 256);
  }
  e->sync_all();  // the staging buffer may still be read by the previous batch
  e->images.ensure(std::max<int64_t>(total, 256));
  for (int i = 0; i < n_img; i++)
    HIP_CHECK(hipMemcpyAsync(e->images.as<uint8_t>() + in[i].img_off, imgs[i].bgr,
                             (size_t)imgs[i].stride * imgs[i].height, hipMemcpyHostToDevice, e->main_stream()));
  return FFD_OK;
}

ffd_status copy_boxes(ffd_engine* e, const std::vector<std::vector<ffd_rect>>& det, ffd_rect* boxes, int32_t* box_img,
                      int32_t max_boxes, int32_t* n_boxes) {
  int32_t n = 0;
  for (size_t k = 0; k < det.size(); k++)
    for (const auto& b : det[k]) {
      if (n < max_boxes) {
        if (boxes) boxes[n] = b;
        if (box_img) box_img[n] = (int32_t)k;
      }
      n++;
    }
  *n_boxes = n;
  (void)e;
  return FFD_OK;
}

template <class F> ffd_status guarded_d(ffd_engine* e, F&& fn) {
  if (!e) return FFD_ERR_INVALID_ARGUMENT;
  try {
    HIP_CHECK(hipSetDevice(e->device));
    return fn();
  } catch (const HipError& x) {
    return fail(e, FFD_ERR_DEVICE, x.what());
  } catch (const std::bad_alloc&) {
    return fail(e, FFD_ERR_OUT_OF_MEMORY, "host allocation failed");
  } catch (const std::exception& x) {
    return fail(e, FFD_ERR_INTERNAL, x.what());
  }
}

}  // namespace

extern "C" {

void ffd_detect_options_init(ffd_detect_options* o) {
  if (o) default_options(o);
}

ffd_status ffd_detect_faces(ffd_engine* e, const ffd_image* imgs, int32_t n_img, const ffd_detect_options* opt,
                            ffd_rect* boxes, int32_t* box_img, int32_t max_boxes, int32_t* n_boxes) {
  return guarded_d(e, [&]() -> ffd_status {
    if (!n_boxes || max_boxes < 0 || (max_boxes > 0 && !boxes)) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    ffd_detect_options o;
    default_options(&o);
    if (opt) o = *opt;
    std::vector<FrameIn> in;
    ffd_status st = upload_frames(e, imgs, n_img, in);
    if (st != FFD_OK) return st;
    std::vector<std::vector<ffd_rect>> det;
    st = detect_batch(e, e->images.as<uint8_t>(), in, o, det, nullptr);
    if (st != FFD_OK) return st;
    return copy_boxes(e, det, boxes, box_img, max_boxes, n_boxes);
  });
}

ffd_status ffd_detect_faces_device(ffd_engine* e, const void* d_images, int64_t image_bytes, int32_t width,
                                   int32_t height, int32_t stride, int32_t n_img, const ffd_detect_options* opt,
                                   ffd_rect* boxes, int32_t* box_img, int32_t max_boxes, int32_t* n_boxes) {
  return guarded_d(e, [&]() -> ffd_status {
    if (!n_boxes || max_boxes < 0 || (max_boxes > 0 && !boxes) || n_img < 0 || (n_img > 0 && !d_images) ||
        width <= 0 || height <= 0 || stride < 3 * width || image_bytes < (int64_t)stride * height)
      return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    ffd_detect_options o;
    default_options(&o);
    if (opt) o = *opt;
    std::vector<FrameIn> in(n_img);
    for (int i = 0; i < n_img; i++) in[i] = FrameIn{(int64_t)i * image_bytes, width, height, stride};
    std::vector<std::vector<ffd_rect>> det;
    ffd_status st = detect_batch(e, static_cast<const uint8_t*>(d_images), in, o, det, nullptr);
    if (st != FFD_OK) return st;
    return copy_boxes(e, det, boxes, box_img, max_boxes, n_boxes);
  });
}

ffd_status ffd_detect_candidates(ffd_engine* e, const ffd_image* img, const ffd_detect_options* opt, ffd_rect* raw,
                                 int32_t cap, int32_t* n_raw) {
  return guarded_d(e, [&]() -> ffd_status {
    if (!img || !n_raw || cap < 0 || (cap > 0 && !raw)) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    ffd_detect_options o;
    default_options(&o);
    if (opt) o = *opt;
    std::vector<FrameIn> in;
    ffd_status st = upload_frames(e, img, 1, in);
    if (st != FFD_OK) return st;
    std::vector<std::vector<ffd_rect>> det, rw;
    st = detect_batch(e, e->images.as<uint8_t>(), in, o, det, &rw);
    if (st != FFD_OK) return st;
    *n_raw = (int32_t)rw[0].size();
    for (int i = 0; i < (int)rw[0].size() && i < cap; i++) raw[i] = rw[0][i];
    return FFD_OK;
  });
}

ffd_status ffd_analyze_images(ffd_engine* e, const ffd_image* imgs, int32_t n_img, const ffd_detect_options* opt,
                              ffd_face* faces, int32_t* face_img, int32_t max_faces, int32_t* n_faces) {
  if (e && e->detector_only) return fail(e, FFD_ERR_INVALID_ARGUMENT, "a detector-only engine (ffd_detector_create) has no forests");
  return guarded_d(e, [&]() -> ffd_status {
    if (!n_faces || max_faces < 0 || (max_faces > 0 && !faces)) return fail(e, FFD_ERR_INVALID_ARGUMENT, "bad arguments");
    ffd_detect_options o;
    default_options(&o);
    if (opt) o = *opt;
    std::vector<FrameIn> in;
    ffd_status st = upload_frames(e, imgs, n_img, in);
    if (st != FFD_OK) return st;
    std::vector<std::vector<ffd_rect>> det;
    st = detect_batch(e, e->images.as<uint8_t>(), in, o, det, nullptr);
    if (st != FFD_OK) return st;
    // analyzeImage: analyzeFace on every detected box (FaceForest.cpp:174-180), as one GPU batch
    std::vector<FaceDesc> fds;
    std::vector<int32_t> owner;
    for (size_t k = 0; k < det.size(); k++)
      for (const auto& b : det[k]) {
        FaceDesc f;
        make_desc(e, in[k].img_off, in[k].w, in[k].h, in[k].stride, b, f);
        fds.push_back(f);
        owner.push_back((int32_t)k);
      }
    *n_faces = (int32_t)fds.size();
    if (fds.empty()) return FFD_OK;
    e->out.ensure(fds.size() * sizeof(FaceOut));
    e->analyze(e->images.as<uint8_t>(), fds, e->out.as<FaceOut>());
    const int32_t n = std::min<int32_t>((int32_t)fds.size(), max_faces);
    if (n > 0)
      HIP_CHECK(hipMemcpyAsync(faces, e->out.p, (size_t)n * sizeof(ffd_face), hipMemcpyDeviceToHost, e->main_stream()));
    HIP_CHECK(hipStreamSynchronize(e->main_stream()));
    for (int32_t i = 0; face_img && i < n; i++) face_img[i] = owner[i];
    return FFD_OK;
  });
}

}  // extern "C"
