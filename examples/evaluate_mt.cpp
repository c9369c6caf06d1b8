// evaluate_mt.cpp — the reference's getFacialFeaturesVotesMT call pattern (src/face_utils.cpp:244-302) through the
// C++ drop-in header: one Forest<MPSample>::evaluateMT call per patch (1,024 for a 125 x 125 face), the vote
// filter over the Leaf* members, then MeanShift::shift per landmark (FaceForest::estimateFacialFeatures,
// src/FaceForest.cpp:74-95).  Written with the reference's global names, as its own code is.
//
// usage: evaluate_mt MODEL FACE.gray WIDTH HEIGHT TREE0 ... TREE(n-1)
//   FACE.gray: raw 8-bit scaled face (WIDTH bytes per row); TREEi: global FFD tree ids (forest*20 + tree).
//        evaluate_mt MODEL --crop IMAGE.bgr WIDTH HEIGHT X Y W H
//   the scaled face and the trees analyzeFace chooses for that box (ffd_get_trace), as bench.py runs it.
// Prints one JSON line: the landmarks (cvRound of the MeanShift modes, sample coordinates), the modes, the vote
// counts, a CRC of the leaf ordinals in the reference's (patch, tree) order, and the timings of the last of
// $FFD_EVAL_REPS (default 3) repetitions of the whole per-face procedure (a fresh ImageSample each): the
// ImageSample, the first evaluateMT call (the grid evaluation), the mean of the other calls, all calls, the
// vote filter and MeanShift; plus the first repetition's first call (cold: first launches, allocations).
// $FFD_EVAL_THREADS=N (default 0) first runs N threads that each build their own ImageSample and their own
// Forest (separate caches, one engine) and walk every patch four times; "thread_crcs" holds each thread's leaf
// CRC (the header serialises the engine calls of distinct objects, detail::engine_call).
// exit: 0 ok, 2 bad arguments, 3 engine not initialised, 4 error.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#define FFD_NO_OPENCV
#include "FaceForest.hpp"

using Clock = std::chrono::steady_clock;
static double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

static uint32_t crc32(const void* data, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  const uint8_t* p = static_cast<const uint8_t*>(data);
  for (size_t i = 0; i < n; i++) {
    c ^= p[i];
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
  }
  return c ^ 0xFFFFFFFFu;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s MODEL FACE.gray WIDTH HEIGHT TREE0 [TREE1 ...]\n", argv[0]);
    return 2;
  }
  const bool crop = std::string(argv[2]) == "--crop";
  if (crop && argc != 10) return 2;
  const char* file = crop ? argv[3] : argv[2];
  int w = std::atoi(argv[crop ? 4 : 3]), h = std::atoi(argv[crop ? 5 : 4]);
  std::vector<uint8_t> px((size_t)w * h * (crop ? 3 : 1));
  std::ifstream f(file, std::ios::binary);
  if (!f.read(reinterpret_cast<char*>(px.data()), (std::streamsize)px.size())) return 2;
  FaceForestOptions opt;
  opt.model_path = argv[1];
  FaceForest ff(opt);
  if (!ff.is_initialized()) {
    std::fprintf(stderr, "FaceForest: %s\n", ff.last_error().c_str());
    return 3;
  }
  std::vector<int> tree_args;
  for (int a = 5; !crop && a < argc; a++) tree_args.push_back(std::atoi(argv[a]));
  try {
    if (crop) {  // analyzeFace on the box; its scaled face and selected trees from the engine's trace
      const cv::Rect box(std::atoi(argv[6]), std::atoi(argv[7]), std::atoi(argv[8]), std::atoi(argv[9]));
      Face face;
      ff.analyzeFace(cv::Mat(h, w, px.data()), box, face);
      int32_t fw = 0, fh = 0, nhp = 0, nmp = 0;
      if (ffd_face_geometry(ff.engine(), box.width, box.height, &fw, &fh, &nhp, &nmp) != FFD_OK) return 4;
      std::vector<uint8_t> gray((size_t)fw * fh);
      std::vector<int32_t> trees(FFD_MAX_TREES, -1);
      ffd_trace tr{};
      tr.face = gray.data();
      tr.trees = trees.data();
      if (ffd_get_trace(ff.engine(), 0, &tr) != FFD_OK) return 4;
      px = gray;
      w = fw;
      h = fh;
      for (int32_t t : trees)
        if (t >= 0) tree_args.push_back(t);
    }
    // the per-face forest the reference composes from the jungle (FaceForest.cpp:239-250)
    std::vector<Forest<MPSample>> jungle;
    for (int i = 0; i < 5; i++) jungle.push_back(ff.ffdForest(i));
    Forest<MPSample> forest;
    forest.setParam(jungle[0].getParam());
    for (int g : tree_args) forest.addTree(jungle.at(g / 20).getTree(g % 20));
    // threads on one engine, each with its own sample and forest (FFD_EVAL_THREADS)
    std::string thread_json;
    const int nthreads = std::getenv("FFD_EVAL_THREADS") ? std::max(0, std::atoi(std::getenv("FFD_EVAL_THREADS"))) : 0;
    if (nthreads > 0) {
      std::vector<Forest<MPSample>> own(nthreads);
      for (auto& fk : own) {  // composed here: getTree() may copy the jungle's tree list
        fk.setParam(jungle[0].getParam());
        for (int g : tree_args) fk.addTree(jungle.at(g / 20).getTree(g % 20));
      }
      // $FFD_EVAL_SHARED=1: every thread works on a copy of ONE forest (one cache), each with its own samples, so
      // the threads replace the cache's grid while others still read the grid they hold
      if (std::getenv("FFD_EVAL_SHARED") && std::atoi(std::getenv("FFD_EVAL_SHARED")))
        for (int k = 1; k < nthreads; k++) own[k] = own[0];
      std::vector<uint32_t> crcs(nthreads, 0);
      std::atomic<int> errors{0};
      std::vector<std::thread> th;
      for (int k = 0; k < nthreads; k++)
        th.emplace_back([&, k] {
          try {
            const int ps = own[k].getParam().getPatchSize(), step = MultiPartEstimatorOption().step_size;
            const int T = own[k].numberOfTrees();
            for (int it = 0; it < 4; it++) {
              ImageSample s(cv::Mat(h, w, px.data(), (size_t)w, 1), std::vector<int>{0, 1, 2}, true);
              std::vector<int32_t> ids;
              for (int x = 0; x < w - ps; x += step)
                for (int y = 0; y < h - ps; y += step) {
                  MPSample m(&s, cv::Rect(x, y, ps, ps));
                  ids.resize(ids.size() + T);
                  own[k].evaluateMT(&m, &ids[ids.size() - T]);
                }
              const uint32_t c = crc32(ids.data(), ids.size() * 4);
              if (it > 0 && c != crcs[k]) errors++;
              crcs[k] = c;
            }
          } catch (const std::exception& e) {
            std::fprintf(stderr, "thread %d: %s\n", k, e.what());
            errors++;
          }
        });
      for (auto& t : th) t.join();
      thread_json = ", \"thread_errors\": " + std::to_string(errors.load()) + ", \"thread_crcs\": [";
      for (int k = 0; k < nthreads; k++) thread_json += (k ? ", " : "") + std::to_string(crcs[k]);
      thread_json += "]";
    }
    const int reps = std::getenv("FFD_EVAL_REPS") ? std::max(1, std::atoi(std::getenv("FFD_EVAL_REPS"))) : 3;
    double cold_first_ms = 0;
    for (int rep = 0; rep < reps; rep++) {
      auto t0 = Clock::now();
      ImageSample sample(cv::Mat(h, w, px.data(), (size_t)w, 1), std::vector<int>{0, 1, 2}, true);
      const double sample_ms = ms_since(t0);
      MultiPartEstimatorOption options;
      const cv::Rect face_bbox(0, 0, w, h);
      const int patch_size = forest.getParam().getPatchSize();
      // getFacialFeaturesVotesMT (face_utils.cpp:255-265): the patch grid, x outer, y inner
      std::vector<MPSample> samples;
      for (int x = face_bbox.x; x < face_bbox.x + face_bbox.width - patch_size; x += options.step_size)
        for (int y = face_bbox.y; y < face_bbox.y + face_bbox.height - patch_size; y += options.step_size)
          samples.push_back(MPSample(&sample, cv::Rect(x, y, patch_size, patch_size)));
      const int num_trees = forest.numberOfTrees();
      std::vector<MPLeaf*> leafs(samples.size() * num_trees);
      // one evaluateMT per patch (face_utils.cpp:267-274), a copy of the forest per call as boost::bind makes
      t0 = Clock::now();
      double first_ms = 0;
      for (size_t i = 0; i < samples.size(); i++) {
        Forest<MPSample> copy = forest;
        copy.evaluateMT(&samples[i], &leafs[i * num_trees]);
        if (i == 0) first_ms = ms_since(t0);
      }
      if (rep == 0) cold_first_ms = first_ms;
      const double all_ms = ms_since(t0);
      // the vote filter (face_utils.cpp:276-301)
      t0 = Clock::now();
      std::vector<std::vector<Vote>> votes(options.num_parts);
      for (size_t i = 0; i < samples.size(); i++) {
        const int offset_x = samples[i].getPatch().x + patch_size / 2;
        const int offset_y = samples[i].getPatch().y + patch_size / 2;
        for (int t = 0; t < num_trees; t++) {
          const MPLeaf* leaf = leafs[i * num_trees + t];
          for (int p = 0; p < options.num_parts; p++) {
            float min_pf = options.min_pf;
            if (p == 0 || p == 7) min_pf *= 1.5;  // probability in outer eye parts
            if (leaf->mp_foreground > options.min_forground && leaf->mp_prob_foreground[p] > min_pf &&
                leaf->mp_parts_variance[p] < options.max_variance && leaf->mp_samples > options.min_samples) {
              Vote v;
              v.pos.x = leaf->mp_parts_offset[p].x + offset_x;
              v.pos.y = leaf->mp_parts_offset[p].y + offset_y;
              v.weight = leaf->mp_foreground;
              v.check = true;
              votes[p].push_back(v);
            }
          }
        }
      }
      const double filter_ms = ms_since(t0);
      // the leaf ordinals in the same order, for the parity check
      std::vector<int32_t> ord(samples.size() * num_trees);
      for (size_t i = 0; i < samples.size(); i++) forest.evaluateMT(&samples[i], &ord[i * num_trees]);
      // MeanShift per landmark (FaceForest.cpp:86-95)
      t0 = Clock::now();
      MeanShiftOption ms_option;
      std::vector<cv::Point> pts(options.num_parts);
      std::vector<float> modes(2 * options.num_parts);
      for (int p = 0; p < options.num_parts; p++) {
        MeanShift::shift(votes[p], pts[p], ms_option);
        MeanShift::mode(votes[p], &modes[2 * p], ms_option.max_iterations, ms_option.kernel_size,
                        ms_option.stopping_criteria);
      }
      const double ms_ms = ms_since(t0) / 2;
      if (rep + 1 < reps) continue;
      std::printf("{\"points\": [");
      for (int p = 0; p < options.num_parts; p++) std::printf(p ? ", [%d, %d]" : "[%d, %d]", pts[p].x, pts[p].y);
      std::printf("], \"modes\": [");
      for (int p = 0; p < options.num_parts; p++) std::printf(p ? ", [%.9g, %.9g]" : "[%.9g, %.9g]", modes[2 * p], modes[2 * p + 1]);
      std::printf("], \"vote_counts\": [");
      for (int p = 0; p < options.num_parts; p++) std::printf(p ? ", %zu" : "%zu", votes[p].size());
      std::printf("], \"leaf_crc\": %u, \"patches\": %zu, \"trees\": %d, \"sample_ms\": %.4f, \"first_call_ms\": %.4f, "
                  "\"other_calls_mean_us\": %.4f, \"all_calls_ms\": %.4f, \"vote_filter_ms\": %.4f, \"meanshift_ms\": %.4f, "
                  "\"cold_first_call_ms\": %.4f, \"reps\": %d%s}\n",
                  crc32(ord.data(), ord.size() * 4), samples.size(), num_trees, sample_ms, first_ms,
                  (all_ms - first_ms) * 1e3 / (double)(samples.size() - 1), all_ms, filter_ms, ms_ms, cold_first_ms, reps,
                  thread_json.c_str());
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "evaluate_mt: %s\n", e.what());
    return 4;
  }
  return 0;
}
