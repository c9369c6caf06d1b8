// bench_host.cpp — the C ABI's host-buffer path timed from C++ (no Python in the loop), through the
// drop-in header: FaceForest::analyzeFaces over a batch of crops (ffd_analyze_faces: pageable host
// images in, host records out, upload chunks overlapping the kernels) and the reference's own call
// pattern, one analyzeFace per call (eval_ffd.cpp:89).
//
// usage: bench_host MODEL CROPS.bgr N WIDTH HEIGHT REPS
//   CROPS.bgr: N raw BGR crops of WIDTH x HEIGHT, back to back; every face is the whole crop.
//   Prints one JSON line: batch faces/s (median of REPS calls), single-face latency (median of 50).
// exit: 0 ok, 2 bad arguments, 3 engine not initialised, 4 analysis error.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <vector>

#define FFD_NO_OPENCV
#include "FaceForest.hpp"

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  if (argc != 7) {
    std::fprintf(stderr, "usage: %s MODEL CROPS.bgr N WIDTH HEIGHT REPS\n", argv[0]);
    return 2;
  }
  const int n = std::atoi(argv[3]), w = std::atoi(argv[4]), h = std::atoi(argv[5]), reps = std::max(1, std::atoi(argv[6]));
  const size_t one = (size_t)w * h * 3;
  std::vector<uint8_t> px(one * n);
  std::ifstream f(argv[2], std::ios::binary);
  if (n < 1 || !f.read(reinterpret_cast<char*>(px.data()), (std::streamsize)px.size())) return 2;
  ffd::FaceForestOptions opt;
  opt.model_path = argv[1];
  ffd::FaceForest ff(opt);
  if (!ff.is_initialized()) {
    std::fprintf(stderr, "FaceForest: %s\n", ff.last_error().c_str());
    return 3;
  }
  std::vector<ffd::Mat> imgs;
  std::vector<ffd::Rect> boxes(n, ffd::Rect(0, 0, w, h));
  for (int i = 0; i < n; i++) imgs.emplace_back(h, w, px.data() + one * i);
  std::vector<ffd::Face> faces;
  try {
    ff.analyzeFaces(imgs, boxes, faces);  // warm-up
    std::vector<double> batch;
    for (int r = 0; r < reps; r++) {
      const double t0 = now_ms();
      ff.analyzeFaces(imgs, boxes, faces);
      batch.push_back(now_ms() - t0);
    }
    ffd::Face face;
    for (int r = 0; r < 5; r++) ff.analyzeFace(imgs[0], boxes[0], face);
    std::vector<double> lat;
    for (int r = 0; r < 50; r++) {
      const double t0 = now_ms();
      ff.analyzeFace(imgs[r % n], boxes[0], face);
      lat.push_back(now_ms() - t0);
    }
    const double bm = median(batch);
    std::printf("{\"batch_faces\": %d, \"batch_ms\": %.3f, \"batch_faces_per_s\": %.1f, \"batch_reps\": %d, "
                "\"latency_ms_median\": %.4f, \"latency_ms_min\": %.4f, \"latency_calls\": 50, "
                "\"check_face0\": [%d, %d]}\n",
                n, bm, n / (bm / 1e3), reps, median(lat), *std::min_element(lat.begin(), lat.end()),
                faces[0].ffd_cordinates[0].x, faces[0].ffd_cordinates[0].y);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "bench_host: %s\n", e.what());
    return 4;
  }
  return 0;
}
