// FaceForest.hpp — header-only C++ drop-in for the reference's FaceForest API
// (/root/reference/include/FaceForest.hpp:21-157) over the C ABI in ffd.h.
//
// Same type and method names as the reference:
//   HeadPoseEstimatorOption, MultiPartEstimatorOption, FaceDetectionOption, FaceForestOptions,
//   Face { headpose, bbox, ffd_cordinates }, FaceForest(FaceForestOptions),
//   FaceForest::analyzeFace(img, bbox, Face&)      (FaceForest.cpp:183-258)
//   FaceForest::analyzeImage(img, boxes, faces)    (FaceForest.cpp:161-181 without detectFace:
//                                                   the Haar detector stays on the caller's side)
// With OpenCV available, Mat / Rect / Point are cv::Mat / cv::Rect / cv::Point; otherwise the
// minimal PODs below.  FaceForestOptions carries the converted model path instead of the
// reference's per-forest tree directories (convert once with ffd_convert).
//
// Errors: like the reference constructor (FaceForest.cpp:23-56) a failed construction leaves
// the object uninitialised (is_initialized() == false, message in last_error()); analyzeFace
// on a bad box throws std::invalid_argument where the reference's CV_Assert throws.
//
// Link: -lffd (face_alignment_cvpr_2012_amd/lib/libffd.so) -lamdhip64.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "ffd.h"

#if defined(FFD_WITH_OPENCV) || (defined(__has_include) && __has_include(<opencv2/core/core.hpp>) && !defined(FFD_NO_OPENCV))
#include <opencv2/core/core.hpp>
#define FFD_HAVE_OPENCV 1
#endif

namespace ffd {

#ifdef FFD_HAVE_OPENCV
using Mat = cv::Mat;
using Rect = cv::Rect;
using Point = cv::Point;
inline const uint8_t* mat_data(const Mat& m) { return m.data; }
inline int mat_step(const Mat& m) { return (int)m.step; }
#else
struct Rect {
  int x = 0, y = 0, width = 0, height = 0;
  Rect() = default;
  Rect(int x_, int y_, int w_, int h_) : x(x_), y(y_), width(w_), height(h_) {}
};
struct Point {
  int x = 0, y = 0;
  Point() = default;
  Point(int x_, int y_) : x(x_), y(y_) {}
};
struct Mat {  // BGR 8UC3 view (cv::Mat data / rows / cols / step)
  const uint8_t* data = nullptr;
  int rows = 0, cols = 0;
  size_t step = 0;
  Mat() = default;
  Mat(int rows_, int cols_, const uint8_t* data_, size_t step_ = 0)
      : data(data_), rows(rows_), cols(cols_), step(step_ ? step_ : (size_t)cols_ * 3) {}
};
inline const uint8_t* mat_data(const Mat& m) { return m.data; }
inline int mat_step(const Mat& m) { return (int)m.step; }
#endif

struct FaceDetectionOption {  // kept for source compatibility; detection is the caller's
  int min_feature_size = 30;
  int min_neighbors = 1;
  float search_scale_factor = 1.3f;
  std::string path_face_cascade;
};

struct HeadPoseEstimatorOption {
  int num_head_pose_labels = 5;
  int step_size = 4;
  float min_foreground_probability = 0.5f;
};

struct MultiPartEstimatorOption {
  int num_parts = 10;
  int step_size = 3;
  int min_samples = 2;
  float min_forground = 0.5f;
  float min_pf = 0.25f;
  float max_variance = 25.f;
};

struct MeanShiftOption {  // include/MeanShift.hpp:16-25
  int kernel_size = 10;
  int max_iterations = 7;
  float stopping_criteria = 0.05f;
};

struct FaceForestOptions {
  std::string model_path;  // FFDMODEL file (replaces hp_forest_param / mp_forest_paths)
  int device = 0;          // HIP device ordinal
  FaceDetectionOption fd_option;
  HeadPoseEstimatorOption hp_option;
  MultiPartEstimatorOption mp_option;
  MeanShiftOption ms_option;
};

struct Face {
  float headpose = 0.f;
  Rect bbox;
  std::vector<Point> ffd_cordinates;  // 10 bbox-relative landmarks (reference spelling)
};

class FaceForest {
 public:
  FaceForest() = default;
  explicit FaceForest(const FaceForestOptions& option) {
    ffd_engine_desc d;
    ffd_engine_desc_init(&d);
    d.model_path = option.model_path.c_str();
    d.device = option.device;
    d.hp_option = {option.hp_option.num_head_pose_labels, option.hp_option.step_size,
                   option.hp_option.min_foreground_probability};
    d.mp_option = {option.mp_option.num_parts,     option.mp_option.step_size, option.mp_option.min_samples,
                   option.mp_option.min_forground, option.mp_option.min_pf,    option.mp_option.max_variance};
    d.ms_option = {option.ms_option.kernel_size, option.ms_option.max_iterations,
                   option.ms_option.stopping_criteria};
    if (ffd_engine_create(&d, &engine_) != FFD_OK) {
      err_ = ffd_last_error(nullptr);
      engine_ = nullptr;
    }
  }
  FaceForest(const FaceForest&) = delete;
  FaceForest& operator=(const FaceForest&) = delete;
  FaceForest(FaceForest&& o) noexcept : engine_(o.engine_), err_(std::move(o.err_)) { o.engine_ = nullptr; }
  virtual ~FaceForest() { ffd_engine_destroy(engine_); }

  bool is_initialized() const { return engine_ != nullptr; }
  std::string last_error() const { return engine_ ? ffd_last_error(engine_) : err_; }

  // FaceForest::analyzeFace (FaceForest.cpp:183-258)
  void analyzeFace(const Mat img, Rect face_bbox, Face& face) {
    std::vector<Face> faces;
    analyzeImage(img, std::vector<Rect>{face_bbox}, faces);
    face = faces.at(0);
  }

  // FaceForest::analyzeImage (FaceForest.cpp:161-181) with the face boxes supplied by the caller;
  // all boxes run as one batch on the GPU.  Appends to `faces` like the reference.
  void analyzeImage(const Mat img, const std::vector<Rect>& boxes, std::vector<Face>& faces) {
    if (!engine_) throw std::runtime_error("FaceForest not initialised: " + err_);
    ffd_image im{mat_data(img), img.cols, img.rows, mat_step(img)};
    std::vector<ffd_rect> r(boxes.size());
    for (size_t i = 0; i < boxes.size(); i++) r[i] = {boxes[i].x, boxes[i].y, boxes[i].width, boxes[i].height};
    std::vector<int32_t> which(boxes.size(), 0);
    std::vector<ffd_face> out(boxes.size());
    const ffd_status st =
        ffd_analyze_faces(engine_, &im, 1, r.data(), which.data(), (int32_t)r.size(), out.data());
    if (st == FFD_ERR_INVALID_ARGUMENT) throw std::invalid_argument(ffd_last_error(engine_));
    if (st != FFD_OK) throw std::runtime_error(ffd_last_error(engine_));
    for (size_t i = 0; i < out.size(); i++) {
      if (out[i].status != FFD_OK) throw std::invalid_argument("face box outside the image");
      Face f;
      f.headpose = out[i].headpose;
      f.bbox = boxes[i];
      for (int k = 0; k < FFD_NUM_LANDMARKS; k++) f.ffd_cordinates.emplace_back(out[i].points[k][0], out[i].points[k][1]);
      faces.push_back(f);
    }
  }

  ffd_engine* engine() const { return engine_; }

 private:
  ffd_engine* engine_ = nullptr;
  std::string err_;
};

}  // namespace ffd

#ifdef FFD_GLOBAL_NAMES  // drop-in: the reference's global names
using ffd::Face;
using ffd::FaceDetectionOption;
using ffd::FaceForest;
using ffd::FaceForestOptions;
using ffd::HeadPoseEstimatorOption;
using ffd::MultiPartEstimatorOption;
#endif
