// analyze_face.cpp — the reference's analyzeFace call contract through the C++ drop-in header
// (include/FaceForest.hpp), as eval_ffd.cpp:89 / demo.cpp:149 use it.
//
// usage: analyze_face MODEL IMAGE.bgr WIDTH HEIGHT X Y W H   analyzeFace on one box
//        analyze_face MODEL IMAGE.bgr WIDTH HEIGHT            analyzeImage (GPU Haar detectFace first)
//   IMAGE.bgr: raw BGR 8UC3 rows (WIDTH*3 bytes each).  Prints "headpose x0 y0 ... x9 y9" per face
//   (analyzeImage: "bx by bw bh headpose x0 y0 ... x9 y9" per detected face).
//   FFD_REPEAT=N: call analyzeFace N times and print the median per-call latency (the reference's
//   one-face-per-call pattern, eval_ffd.cpp:89) to stderr as "latency_ms <median>".
// exit: 0 ok, 2 bad arguments, 3 engine not initialised (e.g. no HIP device), 4 analysis error.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <vector>

#define FFD_NO_OPENCV
#include "FaceForest.hpp"

int main(int argc, char** argv) {
  if (argc != 9 && argc != 5) {
    std::fprintf(stderr, "usage: %s MODEL IMAGE.bgr WIDTH HEIGHT [X Y W H]\n", argv[0]);
    return 2;
  }
  const int w = std::atoi(argv[3]), h = std::atoi(argv[4]);
  std::vector<uint8_t> px((size_t)w * h * 3);
  std::ifstream f(argv[2], std::ios::binary);
  if (!f.read(reinterpret_cast<char*>(px.data()), (std::streamsize)px.size())) {
    std::fprintf(stderr, "cannot read %s\n", argv[2]);
    return 2;
  }
  ffd::FaceForestOptions opt;
  opt.model_path = argv[1];
  ffd::FaceForest ff(opt);
  if (!ff.is_initialized()) {
    std::fprintf(stderr, "FaceForest: %s\n", ff.last_error().c_str());
    return 3;
  }
  if (argc == 5) {
    std::vector<ffd::Face> faces;
    try {
      ff.analyzeImage(ffd::Mat(h, w, px.data()), faces);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "analyzeImage: %s\n", e.what());
      return 4;
    }
    for (const auto& face : faces) {
      std::printf("%d %d %d %d %.9g", face.bbox.x, face.bbox.y, face.bbox.width, face.bbox.height, face.headpose);
      for (const auto& p : face.ffd_cordinates) std::printf(" %d %d", p.x, p.y);
      std::printf("\n");
    }
    return 0;
  }
  ffd::Face face;
  if (const char* rep = std::getenv("FFD_REPEAT")) {
    std::vector<double> ms;
    const ffd::Rect box(std::atoi(argv[5]), std::atoi(argv[6]), std::atoi(argv[7]), std::atoi(argv[8]));
    for (int i = 0; i < std::max(1, std::atoi(rep)); i++) {
      ffd::Face f;
      const auto t0 = std::chrono::steady_clock::now();
      ff.analyzeFace(ffd::Mat(h, w, px.data()), box, f);
      ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(ms.begin(), ms.end());
    std::fprintf(stderr, "latency_ms %.4f\n", ms[ms.size() / 2]);
  }
  try {
    ff.analyzeFace(ffd::Mat(h, w, px.data()), ffd::Rect(std::atoi(argv[5]), std::atoi(argv[6]), std::atoi(argv[7]),
                                                        std::atoi(argv[8])),
                   face);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "analyzeFace: %s\n", e.what());
    return 4;
  }
  std::printf("%.9g", face.headpose);
  for (const auto& p : face.ffd_cordinates) std::printf(" %d %d", p.x, p.y);
  std::printf("\n");
  return 0;
}
