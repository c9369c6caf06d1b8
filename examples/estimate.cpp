// estimate.cpp — the reference's lower-level FaceForest API through the C++ drop-in header:
// ImageSample (ImageSample.cpp:11-20), FaceForest::estimateHeadPose / estimateFacialFeatures
// (static, FaceForest.cpp:60-95) and Forest<S>::evaluateMT (Forest.hpp:80-90), as analyzeFace
// composes them (FaceForest.cpp:207-253).
//
// usage: estimate MODEL FACE.gray WIDTH HEIGHT RX RY RW RH POSE_BIN
//   FACE.gray: raw 8-bit scaled face (WIDTH bytes per row).  Prints three lines:
//   "headpose variance", "x0 y0 ... x9 y9" (pose forest POSE_BIN over the region), and the 15
//   head-pose leaf ordinals of the patch at (RX, RY).
// exit: 0 ok, 2 bad arguments, 3 engine not initialised, 4 estimation error.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <vector>

#define FFD_NO_OPENCV
#include "FaceForest.hpp"

int main(int argc, char** argv) {
  if (argc != 10) {
    std::fprintf(stderr, "usage: %s MODEL FACE.gray WIDTH HEIGHT RX RY RW RH POSE_BIN\n", argv[0]);
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
  try {
    ffd::ImageSample sample(px.data(), w, h, (size_t)w, {0, 1, 2}, true);
    float headpose = 0, variance = 0;
    const ffd::Forest<ffd::HeadPoseSample> hp = ff.headPoseForest();
    ffd::FaceForest::estimateHeadPose(sample, region, hp, opt.hp_option, &headpose, &variance);
    std::printf("%.9g %.9g\n", headpose, variance);
    std::vector<ffd::Point> pts;
    ffd::FaceForest::estimateFacialFeatures(sample, region, ff.ffdForest(std::atoi(argv[9])), opt.mp_option, pts);
    for (size_t i = 0; i < pts.size(); i++) std::printf(i ? " %d %d" : "%d %d", pts[i].x, pts[i].y);
    std::printf("\n");
    ffd::HeadPoseSample patch(&sample, ffd::Rect(region.x, region.y, 31, 31));
    std::vector<int32_t> leafs(hp.numberOfTrees());
    hp.evaluateMT(&patch, leafs.data());
    for (size_t i = 0; i < leafs.size(); i++) std::printf(i ? " %d" : "%d", leafs[i]);
    std::printf("\n");
  } catch (const std::exception& e) {
    std::fprintf(stderr, "estimate: %s\n", e.what());
    return 4;
  }
  return 0;
}
