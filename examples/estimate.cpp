// estimate.cpp — the reference's lower-level FaceForest API through the C++ drop-in header:
// ImageSample (ImageSample.cpp:11-20), FaceForest::estimateHeadPose / estimateFacialFeatures
// (static, FaceForest.cpp:60-95) and Forest<S>::evaluateMT (Forest.hpp:80-90), as analyzeFace
// composes them (FaceForest.cpp:207-253).
//
// usage: estimate MODEL FACE.gray WIDTH HEIGHT RX RY RW RH POSE_BIN [key=value ...]
//   FACE.gray: raw 8-bit scaled face (WIDTH bytes per row).  key=value sets a field of the options
//   passed to the static estimators (hp_step, hp_min_fg, hp_labels, mp_step, mp_parts, mp_min_samples,
//   mp_min_fg, mp_min_pf, mp_max_var); the engine itself keeps the defaults.  Prints four lines:
//   "headpose variance", "x0 y0 ... x(n-1) y(n-1)" (pose forest POSE_BIN over the region), the 15
//   head-pose leaf ordinals of the patch at (RX, RY), and for that patch's FFD leaves (Leaf** form of
//   Forest<MPSample>::evaluateMT) "mp_samples mp_foreground offset[0].x offset[0].y" per tree.
// exit: 0 ok, 2 bad arguments, 3 engine not initialised, 4 estimation error.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#define FFD_NO_OPENCV
#include "FaceForest.hpp"

int main(int argc, char** argv) {
  if (argc < 10) {
    std::fprintf(stderr, "usage: %s MODEL FACE.gray WIDTH HEIGHT RX RY RW RH POSE_BIN [key=value ...]\n", argv[0]);
    return 2;
  }
  const int w = std::atoi(argv[3]), h = std::atoi(argv[4]);
  std::vector<uint8_t> px((size_t)w * h);
  std::ifstream f(argv[2], std::ios::binary);
  if (!f.read(reinterpret_cast<char*>(px.data()), (std::streamsize)px.size())) return 2;
  ffd::FaceForestOptions opt;
  opt.model_path = argv[1];
  ffd::FaceForest ff(opt);
  if (!ff.is_initialized()) {
    std::fprintf(stderr, "FaceForest: %s\n", ff.last_error().c_str());
    return 3;
  }
  const ffd::Rect region(std::atoi(argv[5]), std::atoi(argv[6]), std::atoi(argv[7]), std::atoi(argv[8]));
  ffd::HeadPoseEstimatorOption hpo = opt.hp_option;
  ffd::MultiPartEstimatorOption mpo = opt.mp_option;
  for (int a = 10; a < argc; a++) {
    const char* eq = std::strchr(argv[a], '=');
    if (!eq) return 2;
    const std::string k(argv[a], eq - argv[a]);
    const double v = std::atof(eq + 1);
    if (k == "hp_step") hpo.step_size = (int)v;
    else if (k == "hp_min_fg") hpo.min_foreground_probability = (float)v;
    else if (k == "hp_labels") hpo.num_head_pose_labels = (int)v;
    else if (k == "mp_step") mpo.step_size = (int)v;
    else if (k == "mp_parts") mpo.num_parts = (int)v;
    else if (k == "mp_min_samples") mpo.min_samples = (int)v;
    else if (k == "mp_min_fg") mpo.min_forground = (float)v;
    else if (k == "mp_min_pf") mpo.min_pf = (float)v;
    else if (k == "mp_max_var") mpo.max_variance = (float)v;
    else return 2;
  }
  try {
    ffd::ImageSample sample(px.data(), w, h, (size_t)w, {0, 1, 2}, true);
    float headpose = 0, variance = 0;
    const ffd::Forest<ffd::HeadPoseSample> hp = ff.headPoseForest();
    ffd::FaceForest::estimateHeadPose(sample, region, hp, hpo, &headpose, &variance);
    std::printf("%.9g %.9g\n", headpose, variance);
    std::vector<ffd::Point> pts;
    const ffd::Forest<ffd::MPSample> mp = ff.ffdForest(std::atoi(argv[9]));
    ffd::FaceForest::estimateFacialFeatures(sample, region, mp, mpo, pts);
    for (size_t i = 0; i < pts.size(); i++) std::printf(i ? " %d %d" : "%d %d", pts[i].x, pts[i].y);
    std::printf("\n");
    ffd::HeadPoseSample patch(&sample, ffd::Rect(region.x, region.y, 31, 31));
    std::vector<int32_t> leafs(hp.numberOfTrees());
    hp.evaluateMT(&patch, leafs.data());
    for (size_t i = 0; i < leafs.size(); i++) std::printf(i ? " %d" : "%d", leafs[i]);
    std::printf("\n");
    // the reference's Leaf** form (face_utils.cpp:273-295 reads these members)
    ffd::MPSample mpatch(&sample, ffd::Rect(region.x, region.y, 31, 31));
    std::vector<ffd::MPLeaf*> mleafs(mp.numberOfTrees());
    mp.evaluateMT(&mpatch, mleafs.data());
    for (size_t t = 0; t < mleafs.size(); t++)
      std::printf(t ? " %d %.9g %d %d" : "%d %.9g %d %d", mleafs[t]->mp_samples, mleafs[t]->mp_foreground,
                  mleafs[t]->mp_parts_offset[0].x, mleafs[t]->mp_parts_offset[0].y);
    std::printf("\n");
  } catch (const std::exception& e) {
    std::fprintf(stderr, "estimate: %s\n", e.what());
    return 4;
  }
  return 0;
}
