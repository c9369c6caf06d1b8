// reference_main.cpp — a reference main's setup, unchanged (the include path decides): eval_ffd's configuration
// (src/eval_ffd.cpp:137-174: loadConfigFile for both forests, FaceForestOptions with hp_forest_param /
// mp_forest_param / the cascade path, FaceForest(ff_options)), then analyzeFace on one image (eval_ffd.cpp:89)
// and the static detectFace with a CascadeClassifier (FaceForest.cpp:136-159).
//
// usage: reference_main CONFIG_HEADPOSE CONFIG_FFD CASCADE_XML IMAGE.bgr WIDTH HEIGHT X Y W H
// Prints "headpose x0 y0 ... x9 y9" and then "n_detected" (the static detectFace's box count).
// exit: 0 ok, 1 config not found, 2 bad arguments, 3 FaceForest not initialised, 4 analysis error.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "FaceForest.hpp"

int main(int argc, char** argv) {
  if (argc != 11) {
    std::fprintf(stderr, "usage: %s CONFIG_HP CONFIG_FFD CASCADE IMAGE.bgr W H X Y BW BH\n", argv[0]);
    return 2;
  }
  // Evaluate feature points detector (eval_ffd.cpp:139-174)
  std::string ffd_config_file = argv[2];
  std::string headpose_config_file = argv[1];
  std::string face_cascade = argv[3];

  // Parse configuration files
  ForestParam hp_param, mp_param;
  if (!loadConfigFile(headpose_config_file, hp_param)) return EXIT_FAILURE;
  if (!loadConfigFile(ffd_config_file, mp_param)) return EXIT_FAILURE;

  FaceForestOptions ff_options;
  ff_options.fd_option.path_face_cascade = face_cascade;
  ff_options.hp_forest_param = hp_param;
  ff_options.mp_forest_param = mp_param;

  FaceForest ff(ff_options);
  if (!ff.is_initialized()) {
    std::fprintf(stderr, "FaceForest: %s\n", ff.last_error().c_str());
    return 3;
  }
  const int w = std::atoi(argv[5]), h = std::atoi(argv[6]);
  std::vector<uint8_t> px((size_t)w * h * 3);
  std::ifstream f(argv[4], std::ios::binary);
  if (!f.read(reinterpret_cast<char*>(px.data()), (std::streamsize)px.size())) return 2;
  try {
    cv::Mat img(h, w, CV_8UC3, px.data());
    Face face;
    ff.analyzeFace(img, cv::Rect(std::atoi(argv[7]), std::atoi(argv[8]), std::atoi(argv[9]), std::atoi(argv[10])), face);
    std::printf("%.9g", face.headpose);
    for (const cv::Point& p : face.ffd_cordinates) std::printf(" %d %d", p.x, p.y);
    std::printf("\n");
    cv::CascadeClassifier cascade;
    if (!cascade.load(face_cascade)) return 1;
    std::vector<cv::Rect> boxes;
    FaceForest::detectFace(img, cascade, ff_options.fd_option, boxes);
    std::printf("%zu\n", boxes.size());
  } catch (const std::exception& e) {
    std::fprintf(stderr, "reference_main: %s\n", e.what());
    return 4;
  }
  return 0;
}
