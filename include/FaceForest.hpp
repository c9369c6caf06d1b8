// FaceForest.hpp — header-only C++ drop-in for the reference's FaceForest API
// (/root/reference/include/FaceForest.hpp:21-157) over the C ABI in ffd.h.
//
// Same type and method names as the reference:
//   HeadPoseEstimatorOption, MultiPartEstimatorOption, FaceDetectionOption, FaceForestOptions,
//   Face { headpose, bbox, ffd_cordinates }, FaceForest(FaceForestOptions),
//   FaceForest::analyzeFace(img, bbox, Face&)      (FaceForest.cpp:183-258)
//   FaceForest::analyzeImage(img, faces)           (FaceForest.cpp:161-181: the GPU Haar detector, then
//                                                   analyzeFace on every box, one GPU batch)
//   FaceForest::detectFace(img, boxes)             (FaceForest.cpp:136-159, the model's cascade)
//   FaceForest::analyzeImage(img, boxes, faces)    (the same with the caller's own boxes)
//   FaceForest::estimateHeadPose / estimateFacialFeatures (static, FaceForest.hpp:97-115,
//                                                   FaceForest.cpp:60-95) over an ImageSample
//   ImageSample(img, features, useIntegral)         (ImageSample.cpp:11-20, channels on the GPU)
//   Forest<HeadPoseSample|MPSample>::evaluateMT     (Forest.hpp:80-90; S::Leaf** with the reference's
//                                                   HeadPoseLeaf / MPLeaf members, or model leaf ordinals)
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

#include <algorithm>
#include <cstdint>
#include <map>
#include <memory>
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

struct FaceDetectionOption {  // include/FaceForest.hpp:21-32 (the cascade comes from the converted model)
  int min_feature_size = 30;
  int min_neighbors = 1;
  float search_scale_factor = 1.3f;
  std::string path_face_cascade;  // unused: ffd_convert puts data/haarcascade_frontalface_alt.xml in the model
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

namespace detail {
inline ffd_engine*& current_engine() {  // the most recently constructed FaceForest's engine
  static ffd_engine* e = nullptr;
  return e;
}
}  // namespace detail

// ImageSample (include/ImageSample.hpp, src/ImageSample.cpp:11-20,77-90): the 38 integral feature
// channels of a scaled gray face, extracted by the engine's HIP kernels (ffd_extract_channels).
// img: 8-bit single-channel face (data, rows, cols, step in bytes); features must be {0, 1, 2} and
// useIntegral true (the only configuration the pretrained forests use, data/config_ffd.txt).
class ImageSample {
 public:
  ImageSample(const uint8_t* gray, int cols, int rows, size_t step, const std::vector<int>& features = {0, 1, 2},
              bool useIntegral = true, ffd_engine* engine = nullptr)
      : engine_(engine ? engine : detail::current_engine()), w_(cols), h_(rows) {
    std::vector<int> f(features);
    std::sort(f.begin(), f.end());
    if (f != std::vector<int>({0, 1, 2}) || !useIntegral)
      throw std::invalid_argument("ImageSample: only features {0,1,2} with integral channels are supported");
    if (!engine_) throw std::runtime_error("ImageSample: no FaceForest engine");
    std::vector<uint8_t> packed((size_t)cols * rows);
    for (int y = 0; y < rows; y++)
      for (int x = 0; x < cols; x++) packed[(size_t)y * cols + x] = gray[(size_t)y * step + x];
    ch_.resize((size_t)38 * (rows + 1) * (cols + 1));
    const ffd_status st = ffd_extract_channels(engine_, packed.data(), cols, rows, ch_.data());
    if (st != FFD_OK) throw std::runtime_error(std::string("ImageSample: ") + ffd_last_error(engine_));
  }
  int width() const { return w_; }
  int height() const { return h_; }
  const uint32_t* channels() const { return ch_.data(); }  // [38][rows+1][cols+1]
  ffd_engine* engine() const { return engine_; }

 private:
  ffd_engine* engine_;
  int w_, h_;
  std::vector<uint32_t> ch_;
};

// Leaf payloads (HeadPoseSample.hpp:144-162, MPSample.hpp:137-159), same member names, so the
// reference's callers (face_utils.cpp:223-228, 289-295) read them through Leaf* unchanged.
struct HeadPoseLeaf {
  int hp_nsamples = 0;          // number of patches reached the leaf
  float hp_foreground = 0.f;    // positive patches percentage
  std::vector<int> hp_labels;   // number of patches for each class
};
struct MPLeaf {
  int mp_samples = 0;                      // number of patches reached the leaf
  std::vector<Point> mp_parts_offset;      // vector of facial points
  std::vector<float> mp_parts_variance;    // variance of the votes
  std::vector<float> mp_prob_foreground;   // probability of foreground per each point
  float mp_foreground = 0.f;               // probability of face
};

// HeadPoseSample / MPSample test constructors (HeadPoseSample.hpp:49-54, MPSample.hpp:47-52): a
// 31 x 31 patch of an ImageSample.
struct HeadPoseSample {
  typedef HeadPoseLeaf Leaf;
  const ImageSample* image;
  Rect roi;
  HeadPoseSample(const ImageSample* i, Rect r) : image(i), roi(r) {}
  Rect getPatch() const { return roi; }
};
struct MPSample {
  typedef MPLeaf Leaf;
  const ImageSample* image;
  Rect roi;
  MPSample(const ImageSample* i, Rect r) : image(i), roi(r) {}
  Rect getPatch() const { return roi; }
};
template <class S> struct ForestKind;
template <> struct ForestKind<HeadPoseSample> {
  static constexpr int value = FFD_FOREST_HEADPOSE;
  typedef ffd_headpose_leaf Raw;
  static void fill(const Raw& r, HeadPoseLeaf& l) {
    l.hp_nsamples = r.hp_nsamples;
    l.hp_foreground = r.hp_foreground;
    l.hp_labels.assign(r.hp_labels, r.hp_labels + FFD_NUM_HP_LABELS_MAX);
  }
};
template <> struct ForestKind<MPSample> {
  static constexpr int value = FFD_FOREST_FFD;
  typedef ffd_mp_leaf Raw;
  static void fill(const Raw& r, MPLeaf& l) {
    l.mp_samples = r.mp_samples;
    l.mp_foreground = r.mp_foreground;
    l.mp_parts_offset.clear();
    for (int i = 0; i < FFD_NUM_LANDMARKS; i++) l.mp_parts_offset.emplace_back(r.mp_parts_offset[i][0], r.mp_parts_offset[i][1]);
    l.mp_parts_variance.assign(r.mp_parts_variance, r.mp_parts_variance + FFD_NUM_LANDMARKS);
    l.mp_prob_foreground.assign(r.mp_prob_foreground, r.mp_prob_foreground + FFD_NUM_LANDMARKS);
  }
};

// Forest<S> (include/Forest.hpp): a list of the engine's trees; evaluateMT walks every tree for
// one patch on the GPU (Forest.hpp:80-90).  Two forms: leaf ordinals (the converted model's order),
// or the reference's `S::Leaf**` (Forest.hpp:80: leafs[t] = the leaf tree t reached), whose payloads
// (ffd_forest_leaves) the Forest owns and keeps for its lifetime, so the pointers stay valid as the
// reference's tree-owned leaves do.
template <class S> class Forest {
 public:
  typedef typename S::Leaf Leaf;
  Forest(ffd_engine* e, std::vector<int32_t> trees) : engine_(e), trees_(std::move(trees)) {}
  int numberOfTrees() const { return (int)trees_.size(); }
  const std::vector<int32_t>& treeIds() const { return trees_; }
  ffd_engine* engine() const { return engine_; }
  void evaluateMT(const S* sample, int32_t* leafs) const {
    const ImageSample& im = *sample->image;
    const int32_t xy[2] = {sample->roi.x, sample->roi.y};
    const ffd_status st = ffd_forest_eval_leaves(engine_, ForestKind<S>::value, im.channels(), im.width(),
                                                 im.height(), xy, 1, trees_.data(), (int32_t)trees_.size(), leafs);
    if (st != FFD_OK) throw std::invalid_argument(ffd_last_error(engine_));
  }
  // Forest<S>::evaluateMT(const S* sample, typename S::Leaf** leafs) const (Forest.hpp:80-90)
  void evaluateMT(const S* sample, Leaf** leafs) const {
    std::vector<int32_t> ids(trees_.size());
    evaluateMT(sample, ids.data());
    for (size_t t = 0; t < ids.size(); t++) leafs[t] = &leaf(ids[t]);
  }
  // the payload of a leaf ordinal (cached; the reference: TreeNode::getLeaf, TreeNode.hpp:61-66)
  Leaf& leaf(int32_t ordinal) const {
    auto it = leaves_.find(ordinal);
    if (it != leaves_.end()) return *it->second;
    typename ForestKind<S>::Raw raw;
    const ffd_status st = ffd_forest_leaves(engine_, ForestKind<S>::value, &ordinal, 1, &raw);
    if (st != FFD_OK) throw std::invalid_argument(ffd_last_error(engine_));
    std::unique_ptr<Leaf> l(new Leaf());
    ForestKind<S>::fill(raw, *l);
    return *(leaves_[ordinal] = std::move(l));
  }

 private:
  ffd_engine* engine_;
  std::vector<int32_t> trees_;
  mutable std::map<int32_t, std::unique_ptr<Leaf>> leaves_;
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
    if (engine_) detail::current_engine() = engine_;
    fd_option_ = option.fd_option;
  }
  FaceForest(const FaceForest&) = delete;
  FaceForest& operator=(const FaceForest&) = delete;
  FaceForest(FaceForest&& o) noexcept : engine_(o.engine_), err_(std::move(o.err_)), fd_option_(o.fd_option_) {
    o.engine_ = nullptr;
  }
  virtual ~FaceForest() {
    if (engine_ && detail::current_engine() == engine_) detail::current_engine() = nullptr;
    ffd_engine_destroy(engine_);
  }

  bool is_initialized() const { return engine_ != nullptr; }
  std::string last_error() const { return engine_ ? ffd_last_error(engine_) : err_; }

  // FaceForest::analyzeFace (FaceForest.cpp:183-258)
  void analyzeFace(const Mat img, Rect face_bbox, Face& face) {
    std::vector<Face> faces;
    analyzeImage(img, std::vector<Rect>{face_bbox}, faces);
    face = faces.at(0);
  }

  // FaceForest::detectFace (FaceForest.cpp:136-159) with this object's fd_option, on the GPU.
  void detectFace(const Mat img, std::vector<Rect>& faces_bboxes) {
    if (!engine_) throw std::runtime_error("FaceForest not initialised: " + err_);
    ffd_image im{mat_data(img), img.cols, img.rows, mat_step(img)};
    const ffd_detect_options o = detect_options();
    std::vector<ffd_rect> r(64);
    int32_t n = 0;
    for (int pass = 0; pass < 2; pass++) {
      const ffd_status st = ffd_detect_faces(engine_, &im, 1, &o, r.data(), nullptr, (int32_t)r.size(), &n);
      if (st != FFD_OK) throw std::runtime_error(ffd_last_error(engine_));
      if (n <= (int32_t)r.size()) break;
      r.resize(n);
    }
    faces_bboxes.clear();
    for (int32_t i = 0; i < n; i++) faces_bboxes.emplace_back(r[i].x, r[i].y, r[i].width, r[i].height);
  }

  // FaceForest::analyzeImage (FaceForest.cpp:161-181): detectFace, then analyzeFace on every box (one
  // GPU batch).  Appends to `faces` like the reference; faces with no usable analysis are skipped
  // only if the reference would throw for them (never for detector boxes, which lie in the image).
  void analyzeImage(const Mat img, std::vector<Face>& faces) {
    if (!engine_) throw std::runtime_error("FaceForest not initialised: " + err_);
    ffd_image im{mat_data(img), img.cols, img.rows, mat_step(img)};
    const ffd_detect_options o = detect_options();
    std::vector<ffd_face> out(64);
    int32_t n = 0;
    for (int pass = 0; pass < 2; pass++) {
      const ffd_status st = ffd_analyze_images(engine_, &im, 1, &o, out.data(), nullptr, (int32_t)out.size(), &n);
      if (st != FFD_OK) throw std::runtime_error(ffd_last_error(engine_));
      if (n <= (int32_t)out.size()) break;
      out.resize(n);
    }
    for (int32_t i = 0; i < n; i++) {
      if (out[i].status != FFD_OK)
        throw std::invalid_argument("face " + std::to_string(i) + ": " + ffd_status_string(out[i].status));
      Face f;
      f.headpose = out[i].headpose;
      f.bbox = Rect(out[i].bbox.x, out[i].bbox.y, out[i].bbox.width, out[i].bbox.height);
      for (int k = 0; k < FFD_NUM_LANDMARKS; k++) f.ffd_cordinates.emplace_back(out[i].points[k][0], out[i].points[k][1]);
      faces.push_back(f);
    }
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
      if (out[i].status != FFD_OK)
        throw std::invalid_argument("face " + std::to_string(i) + ": " + ffd_status_string(out[i].status));
      Face f;
      f.headpose = out[i].headpose;
      f.bbox = boxes[i];
      for (int k = 0; k < FFD_NUM_LANDMARKS; k++) f.ffd_cordinates.emplace_back(out[i].points[k][0], out[i].points[k][1]);
      faces.push_back(f);
    }
  }

  // analyzeFace over many images at once (box i on imgs[i]; the reference calls analyzeFace per face,
  // eval_ffd.cpp:89): one GPU batch through ffd_analyze_faces, whose image upload overlaps the
  // kernels chunk by chunk.  Replaces `faces` (one Face per box, in order).
  void analyzeFaces(const std::vector<Mat>& imgs, const std::vector<Rect>& boxes, std::vector<Face>& faces) {
    if (!engine_) throw std::runtime_error("FaceForest not initialised: " + err_);
    if (imgs.size() != boxes.size()) throw std::invalid_argument("analyzeFaces: one box per image");
    std::vector<ffd_image> im(imgs.size());
    std::vector<ffd_rect> r(boxes.size());
    for (size_t i = 0; i < imgs.size(); i++) {
      im[i] = ffd_image{mat_data(imgs[i]), imgs[i].cols, imgs[i].rows, mat_step(imgs[i])};
      r[i] = {boxes[i].x, boxes[i].y, boxes[i].width, boxes[i].height};
    }
    out_.resize(boxes.size());
    const ffd_status st = ffd_analyze_faces(engine_, im.data(), (int32_t)im.size(), r.data(), nullptr,
                                            (int32_t)r.size(), out_.data());
    if (st == FFD_ERR_INVALID_ARGUMENT) throw std::invalid_argument(ffd_last_error(engine_));
    if (st != FFD_OK) throw std::runtime_error(ffd_last_error(engine_));
    faces.resize(out_.size());
    for (size_t i = 0; i < out_.size(); i++) {
      if (out_[i].status != FFD_OK)
        throw std::invalid_argument("face " + std::to_string(i) + ": " + ffd_status_string(out_[i].status));
      Face& f = faces[i];
      f.headpose = out_[i].headpose;
      f.bbox = boxes[i];
      f.ffd_cordinates.resize(FFD_NUM_LANDMARKS);
      for (int k = 0; k < FFD_NUM_LANDMARKS; k++) f.ffd_cordinates[k] = Point(out_[i].points[k][0], out_[i].points[k][1]);
    }
  }

  // The engine's forests: the head-pose forest (15 trees) and pose forest i of the FFD jungle
  // (m_mp_jungle[i], 20 trees, global ids i*20 .. i*20+19).
  Forest<HeadPoseSample> headPoseForest() const {
    std::vector<int32_t> t(15);
    for (int i = 0; i < 15; i++) t[i] = i;
    return Forest<HeadPoseSample>(engine_, t);
  }
  Forest<MPSample> ffdForest(int pose_bin) const {
    std::vector<int32_t> t(20);
    for (int i = 0; i < 20; i++) t[i] = pose_bin * 20 + i;
    return Forest<MPSample>(engine_, t);
  }

  // FaceForest::estimateHeadPose (static, FaceForest.cpp:60-72) with the call's options (step_size,
  // num_head_pose_labels, min_foreground_probability), as getHeadPoseVotesMT uses them.
  static void estimateHeadPose(const ImageSample& sample, const Rect& face_bbox, const Forest<HeadPoseSample>& forest,
                               HeadPoseEstimatorOption options, float* headpose, float* variance) {
    const ffd_rect r{face_bbox.x, face_bbox.y, face_bbox.width, face_bbox.height};
    const ffd_headpose_option o{options.num_head_pose_labels, options.step_size, options.min_foreground_probability};
    const ffd_status st = ffd_estimate_headpose(forest.engine(), sample.channels(), sample.width(), sample.height(), &r,
                                                &o, headpose, variance);
    if (st != FFD_OK) throw std::invalid_argument(ffd_last_error(forest.engine()));
  }

  // FaceForest::estimateFacialFeatures (static, FaceForest.cpp:74-95) with the call's
  // MultiPartEstimatorOption (every field, getFacialFeaturesVotesMT); a default MeanShiftOption as in
  // the reference.  Landmarks in sample coordinates (cvRound of the MeanShift modes), num_parts of them.
  static void estimateFacialFeatures(const ImageSample& sample, const Rect face_bbox, const Forest<MPSample>& forest,
                                     MultiPartEstimatorOption options, std::vector<Point>& ffd_cordinates) {
    const ffd_rect r{face_bbox.x, face_bbox.y, face_bbox.width, face_bbox.height};
    const ffd_multipart_option o{options.num_parts, options.step_size,  options.min_samples, options.min_forground,
                                 options.min_pf,    options.max_variance, 0};
    int32_t pts[FFD_NUM_LANDMARKS * 2];
    const ffd_status st = ffd_estimate_facial_features(forest.engine(), sample.channels(), sample.width(), sample.height(),
                                                       &r, forest.treeIds().data(), forest.numberOfTrees(), &o, pts);
    if (st != FFD_OK) throw std::invalid_argument(ffd_last_error(forest.engine()));
    ffd_cordinates.clear();
    for (int i = 0; i < options.num_parts && i < FFD_NUM_LANDMARKS; i++) ffd_cordinates.emplace_back(pts[2 * i], pts[2 * i + 1]);
  }

  ffd_engine* engine() const { return engine_; }

 private:
  ffd_detect_options detect_options() const {
    ffd_detect_options o;
    ffd_detect_options_init(&o);
    o.min_feature_size = fd_option_.min_feature_size;
    o.min_neighbors = fd_option_.min_neighbors;
    o.search_scale_factor = fd_option_.search_scale_factor;
    return o;
  }
  ffd_engine* engine_ = nullptr;
  std::string err_;
  FaceDetectionOption fd_option_;
  std::vector<ffd_face> out_;  // analyzeFaces' result records (reused across calls)
};

}  // namespace ffd

#ifdef FFD_GLOBAL_NAMES  // drop-in: the reference's global names
using ffd::Face;
using ffd::FaceDetectionOption;
using ffd::FaceForest;
using ffd::FaceForestOptions;
using ffd::Forest;
using ffd::HeadPoseSample;
using ffd::ImageSample;
using ffd::MPSample;
using ffd::HeadPoseEstimatorOption;
using ffd::MultiPartEstimatorOption;
#endif
