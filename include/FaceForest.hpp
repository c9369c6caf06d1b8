// FaceForest.hpp — header-only C++ drop-in for the reference's FaceForest API
// (/root/reference/include/FaceForest.hpp:21-157) over the C ABI in ffd.h.
//
// Same type and method names as the reference:
//   ForestParam                                     (Constants.hpp:24-60), loadConfigFile, loadAnnotations,
//                                                   FaceAnnotation, intersect, enlargeFace (face_utils.cpp:18-181,
//                                                   325-346), Vote (face_utils.hpp:34-42)
//   HeadPoseEstimatorOption, MultiPartEstimatorOption, FaceDetectionOption, FaceForestOptions (with
//   hp_forest_param / mp_forest_param / mp_forest_paths), Face { headpose, bbox, ffd_cordinates },
//   FaceForest(FaceForestOptions)                   (FaceForest.cpp:15-58: the tree directories of the options are
//                                                   converted once by ffd_model_convert and cached; or a converted
//                                                   model via the extension field model_path / $FFD_MODEL)
//   FaceForest::analyzeFace(img, bbox, Face&)       (FaceForest.cpp:183-258)
//   FaceForest::analyzeImage(img, faces)            (FaceForest.cpp:161-181: the GPU Haar detector, then
//                                                   analyzeFace on every box, one GPU batch)
//   FaceForest::detectFace(img, cascade, fd_option, boxes) (static, FaceForest.cpp:136-159)
//   FaceForest::estimateHeadPose / estimateFacialFeatures (static, FaceForest.hpp:97-115, FaceForest.cpp:60-95)
//   ImageSample(img, features, use_integral)        (ImageSample.cpp:11-20: the channels computed on the GPU and
//                                                   kept there, ffd_sample_create)
//   Forest<HeadPoseSample|MPSample>                 (Forest.hpp: load, evaluateMT(const S*, S::Leaf**),
//                                                   numberOfTrees, getTree / addTree / cleanForest / setParam)
//   MeanShift::shift                                (MeanShift.hpp:41-76, on the GPU)
//   loadImage, getHeadPoseVotesMT, getFacialFeaturesVotesMT, areaUnderCurve (face_utils.hpp), the Constants.hpp
//   identifiers, Tree<MPSample>(samples, param, rng, save_path) with MPSample's training constructor (grown on the
//   GPU, ffd_train_mp_tree_patches), CascadeClassifier::load + the static detectFace with that classifier
// With OpenCV available, Mat / Rect / Point / CascadeClassifier are OpenCV's; otherwise minimal stand-ins with
// OpenCV's signatures (no OpenCV is installed where this was built, so the OpenCV branch is uncompiled here).
// The names are global, as the reference declares them; the forwarding headers of this directory (Constants.hpp,
// face_utils.hpp, MeanShift.hpp, Forest.hpp, Tree.hpp, ImageSample.hpp, MPSample.hpp, HeadPoseSample.hpp) give a
// reference source its own include set.  FFD_NO_GLOBAL_NAMES keeps them in namespace ffd only.
//
// Forest<S>::evaluateMT, the reference's per-patch call (face_utils.cpp:210-216, 267-274: one thread-pool task
// per patch, the Forest bound BY VALUE), evaluates on the GPU: the first call for an image sample walks every
// tree for the whole patch grid that contains the requested patch (step 3 for MPSample, 4 for HeadPoseSample,
// the estimators' defaults; Forest::setGridStep changes it) in one launch over the device-resident sample
// (ffd_sample_eval_grid), and the later calls of that sample — from any copy of the Forest, from any thread —
// read their leaves from that result.  A patch off the grid is one launch of its own (ffd_sample_eval_leaves).
// The leaves are exactly the ones Tree<S>::evaluateMT reaches; only when they are computed differs.
//
// Errors: like the reference constructor (FaceForest.cpp:23-56) a failed construction leaves the object
// uninitialised (is_initialized() == false, message in last_error()); analyzeFace on a bad box throws
// std::invalid_argument where the reference's CV_Assert throws.
//
// Link: -lffd (face_alignment_cvpr_2012_amd/lib/libffd.so) -lamdhip64.
#pragma once

#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <deque>
#include <fstream>
#include <memory>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "ffd.h"

#if defined(FFD_WITH_OPENCV) || (defined(__has_include) && __has_include(<opencv2/core/core.hpp>) && !defined(FFD_NO_OPENCV))
#include <opencv2/core/core.hpp>
#include <opencv2/highgui/highgui.hpp>
#include <opencv2/objdetect/objdetect.hpp>
#define FFD_HAVE_OPENCV 1
#endif

namespace ffd {

#ifdef FFD_HAVE_OPENCV
using Mat = cv::Mat;
using Rect = cv::Rect;
using Point = cv::Point;
using CascadeClassifier = cv::CascadeClassifier;
inline const uint8_t* mat_data(const Mat& m) { return m.data; }
inline int mat_step(const Mat& m) { return (int)m.step; }
using Point2f = cv::Point2f;
using cv::norm;
#else
// Without OpenCV: the few cv::Mat / Rect / Point members the reference's mains and FaceForest use, with
// OpenCV's signatures (the cv:: names below alias these).
#ifndef CV_8UC1
#define CV_8UC1 0
#endif
#ifndef CV_8UC3
#define CV_8UC3 16
#endif
struct Rect {
  int x = 0, y = 0, width = 0, height = 0;
  Rect() = default;
  Rect(int x_, int y_, int w_, int h_) : x(x_), y(y_), width(w_), height(h_) {}
  bool operator==(const Rect& o) const { return x == o.x && y == o.y && width == o.width && height == o.height; }
};
struct Point {
  int x = 0, y = 0;
  Point() = default;
  Point(int x_, int y_) : x(x_), y(y_) {}
  Point& operator+=(const Point& o) { x += o.x; y += o.y; return *this; }
  Point& operator*=(float s) {  // saturate_cast<int> of the product: cvRound (half to even)
    x = (int)std::nearbyint(x * s);
    y = (int)std::nearbyint(y * s);
    return *this;
  }
  bool operator==(const Point& o) const { return x == o.x && y == o.y; }
};
inline Point operator-(const Point& a, const Point& b) { return Point(a.x - b.x, a.y - b.y); }
inline Point operator+(const Point& a, const Point& b) { return Point(a.x + b.x, a.y + b.y); }
struct Point2f {
  float x = 0.f, y = 0.f;
  Point2f() = default;
  Point2f(float x_, float y_) : x(x_), y(y_) {}
};
inline Point2f operator-(const Point2f& a, const Point2f& b) { return Point2f(a.x - b.x, a.y - b.y); }
inline double norm(const Point& p) { return std::sqrt((double)p.x * p.x + (double)p.y * p.y); }
inline double norm(const Point2f& p) { return std::sqrt((double)p.x * p.x + (double)p.y * p.y); }
// cv::Mat stand-in: an 8-bit BGR (CV_8UC3) or gray (CV_8UC1) image, a view of caller memory (the OpenCV
// constructor Mat(rows, cols, type, data, step)) or owning its pixels (Mat(rows, cols, type), loadImage);
// img(rect) is a view of the ROI as in OpenCV.
struct Mat {
  uint8_t* data = nullptr;
  int rows = 0, cols = 0;
  size_t step = 0;
  int cn = 3;
  std::shared_ptr<std::vector<uint8_t>> own;
  Mat() = default;
  Mat(int rows_, int cols_, int type, void* data_, size_t step_ = 0)
      : data(static_cast<uint8_t*>(data_)), rows(rows_), cols(cols_), cn(channels_of(type)) {
    step = step_ ? step_ : (size_t)cols_ * cn;
  }
  Mat(int rows_, int cols_, int type) : rows(rows_), cols(cols_), cn(channels_of(type)) {
    step = (size_t)cols_ * cn;
    own = std::make_shared<std::vector<uint8_t>>(step * (size_t)std::max(rows_, 0));
    data = own->data();
  }
  // (earlier spelling of this header: rows, cols, data, step, channels)
  Mat(int rows_, int cols_, const uint8_t* data_, size_t step_ = 0, int channels_ = 3)
      : data(const_cast<uint8_t*>(data_)), rows(rows_), cols(cols_),
        step(step_ ? step_ : (size_t)cols_ * channels_), cn(channels_) {}
  int channels() const { return cn; }
  int type() const { return cn == 1 ? CV_8UC1 : CV_8UC3; }
  bool empty() const { return !data || rows <= 0 || cols <= 0; }
  Mat operator()(const Rect& r) const {
    if (r.x < 0 || r.y < 0 || r.width < 0 || r.height < 0 || r.x + r.width > cols || r.y + r.height > rows)
      throw std::out_of_range("Mat: ROI outside the image");
    Mat m(*this);
    m.data = data + (size_t)r.y * step + (size_t)r.x * cn;
    m.rows = r.height;
    m.cols = r.width;
    return m;
  }
  Mat clone() const {
    Mat m(rows, cols, type());
    for (int y = 0; y < rows; y++) std::memcpy(m.data + (size_t)y * m.step, data + (size_t)y * step, (size_t)cols * cn);
    return m;
  }
  static int channels_of(int type) {
    if (type != CV_8UC1 && type != CV_8UC3) throw std::invalid_argument("Mat: only CV_8UC1 / CV_8UC3 images");
    return type == CV_8UC1 ? 1 : 3;
  }
};
inline const uint8_t* mat_data(const Mat& m) { return m.data; }
inline int mat_step(const Mat& m) { return (int)m.step; }
#endif

// ---------------------------------------------------------------- parameters --
struct ForestParam {  // include/Constants.hpp:24-60
  int max_depth = 0;          // tree stopping criteria
  int min_patches = 0;        // tree stopping criteria
  int ntests = 0;             // number of tests to find the optimal split
  int ntrees = 0;             // number of trees per forest
  int nimages = 0;            // number of images per class
  int npatches = 0;           // number of patches per image
  int face_size = 0;          // face size in pixels
  float patch_size_ratio = 0; // patch size ratio
  std::string tree_path;      // path to load or save the trees
  std::string image_path;     // path to load images
  std::vector<int> features;  // feature channels
  int getPatchSize() { return static_cast<int>(std::round(face_size * patch_size_ratio)); }
};

// Class identifiers (include/Constants.hpp:61-67)
static const float TRAIN_IMAGES_PERCENTAGE = 0.9f;
static const int NUM_HEADPOSE_CLASSES = 5;
static const float NORM_HEADPOSE_VARIANCE_FACTOR = 0.05f;
static const float PATCH_CLOSE_TO_FEATURE = 0.09f;

// loadConfigFile (face_utils.cpp:50-140): (caption line, value line) pairs in a fixed order; the reference's
// defaults when the file cannot be opened (and false).
inline bool loadConfigFile(std::string path, ForestParam& param) {
  std::ifstream f(path);
  if (f.is_open()) {
    std::string line;
    auto value = [&]() {
      std::getline(f, line);
      std::getline(f, line);
      return line;
    };
    param.image_path = value();
    param.tree_path = value();
    param.ntrees = std::stoi(value());
    param.ntests = std::stoi(value());
    param.max_depth = std::stoi(value());
    param.min_patches = std::stoi(value());
    param.nimages = std::stoi(value());
    param.npatches = std::stoi(value());
    param.face_size = std::stoi(value());
    param.patch_size_ratio = std::stof(value());
    std::istringstream ss(value());
    std::string tok;
    while (std::getline(ss, tok, ' ')) param.features.push_back((int)std::stof(tok));
    return true;
  }
  param.max_depth = 15;
  param.min_patches = 20;
  param.ntests = 250;
  param.ntrees = 10;
  param.nimages = 500;
  param.npatches = 200;
  param.face_size = 100;
  param.patch_size_ratio = 0.25f;
  return false;
}

struct FaceAnnotation {  // include/face_utils.hpp:23-29
  std::vector<Point> parts;
  std::string url;
  Rect bbox;
  int pose = 0;
};

// loadAnnotations (face_utils.cpp:143-181): "url x y w h pose n x0 y0 ..." per line, '#' lines skipped.
inline bool loadAnnotations(std::string path, std::vector<FaceAnnotation>& annotations) {
  std::ifstream f(path);
  if (!f.is_open()) return false;
  std::string line;
  while (std::getline(f, line)) {
    std::vector<std::string> s;
    std::string tok;
    std::istringstream ss(line);
    while (std::getline(ss, tok, ' ')) s.push_back(tok);
    if (!line.empty() && line.back() == ' ') s.push_back("");
    if (s.empty() || s[0] == "#") continue;
    FaceAnnotation a;
    a.url = s.at(0);
    a.bbox = Rect(std::stoi(s.at(1)), std::stoi(s.at(2)), std::stoi(s.at(3)), std::stoi(s.at(4)));
    a.pose = std::stoi(s.at(5));
    const int n = std::stoi(s.at(6));
    for (int i = 0; i < n; i++) a.parts.push_back(Point(std::stoi(s.at(7 + 2 * i)), std::stoi(s.at(8 + 2 * i))));
    annotations.push_back(a);
  }
  return true;
}

// intersect (face_utils.cpp:325-346)
inline Rect intersect(const Rect r1, const Rect r2) {
  Rect i;
  i.x = (r1.x < r2.x) ? r2.x : r1.x;
  i.y = (r1.y < r2.y) ? r2.y : r1.y;
  i.width = ((r1.x + r1.width < r2.x + r2.width) ? r1.x + r1.width : r2.x + r2.width) - i.x;
  i.height = ((r1.y + r1.height < r2.y + r2.height) ? r1.y + r1.height : r2.y + r2.height) - i.y;
  if (i.width <= 0 || i.height <= 0) i = Rect(0, 0, 0, 0);
  return i;
}

// enlargeFace (face_utils.cpp:30-48)
inline void enlargeFace(Mat img, Rect& enlarge_bbox, FaceAnnotation& annotation) {
  const Point offset((int)(annotation.bbox.width * 0.1), (int)(annotation.bbox.height * 0.1));
  const Rect aux(annotation.bbox.x - offset.x, annotation.bbox.y - offset.y, annotation.bbox.width + offset.x * 2,
                 annotation.bbox.height + offset.y * 2);
  enlarge_bbox = intersect(aux, Rect(0, 0, img.cols, img.rows));
  annotation.bbox = Rect(0, 0, enlarge_bbox.width, enlarge_bbox.height);
  for (auto& p : annotation.parts) p += offset;
}

// loadImage (face_utils.cpp:18-28): the file `name` in the directory of `path`, as an 8-bit BGR image; an empty
// Mat when it cannot be read.  With OpenCV this is cv::imread; without it (image decoding is outside the
// engine) binary PPM (P6) and PGM (P5) files are read, which is what the bundled tools write.
inline Mat loadImage(std::string path, std::string name) {
  const std::size_t pos = path.rfind("/") + 1;
  const std::string filename = path.substr(0, pos) + name;
#ifdef FFD_HAVE_OPENCV
  return cv::imread(filename, 1);  // IMREAD_COLOR
#else
  std::ifstream f(filename, std::ios::binary);
  if (!f) return Mat();
  auto token = [&]() {
    std::string t;
    char c;
    while (f.get(c)) {
      if (c == '#') { std::string line; std::getline(f, line); continue; }
      if (std::isspace((unsigned char)c)) { if (!t.empty()) break; continue; }
      t.push_back(c);
    }
    return t;
  };
  const std::string magic = token();
  if (magic != "P6" && magic != "P5") return Mat();
  int w = 0, h = 0, mx = 0;
  try {
    w = std::stoi(token());
    h = std::stoi(token());
    mx = std::stoi(token());
  } catch (...) {
    return Mat();
  }
  if (w <= 0 || h <= 0 || mx != 255) return Mat();
  const int cn = magic == "P6" ? 3 : 1;
  std::vector<uint8_t> px((size_t)w * h * cn);
  if (!f.read(reinterpret_cast<char*>(px.data()), (std::streamsize)px.size())) return Mat();
  Mat m(h, w, CV_8UC3);
  for (size_t i = 0; i < (size_t)w * h; i++) {
    uint8_t* d = m.data + 3 * i;
    if (cn == 3) { d[0] = px[3 * i + 2]; d[1] = px[3 * i + 1]; d[2] = px[3 * i]; }  // RGB -> BGR
    else d[0] = d[1] = d[2] = px[i];
  }
  return m;
#endif
}

struct FaceDetectionOption {  // include/FaceForest.hpp:21-32
  int min_feature_size = 30;
  int min_neighbors = 1;
  float search_scale_factor = 1.3f;
  std::string path_face_cascade;
};

struct HeadPoseEstimatorOption {  // include/FaceForest.hpp:34-43
  int num_head_pose_labels = 5;
  int step_size = 4;
  float min_foreground_probability = 0.5f;
};

struct MultiPartEstimatorOption {  // include/FaceForest.hpp:45-58
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

struct FaceForestOptions {  // include/FaceForest.hpp:60-68
  ForestParam hp_forest_param;
  ForestParam mp_forest_param;
  FaceDetectionOption fd_option;
  HeadPoseEstimatorOption hp_option;
  MultiPartEstimatorOption mp_option;
  std::vector<std::string> mp_forest_paths;
  // extensions (not in the reference)
  std::string model_path;  // a converted FFDMODEL file instead of the tree directories ($FFD_MODEL)
  int device = 0;          // HIP device ordinal
  MeanShiftOption ms_option;
};

struct Face {  // include/FaceForest.hpp:70-75
  float headpose = 0.f;
  Rect bbox;
  std::vector<Point> ffd_cordinates;  // 10 bbox-relative landmarks (reference spelling)
};

struct Vote {  // include/face_utils.hpp:34-42
  Point pos;
  float weight = 0.f;
  bool check = false;
};

namespace detail {
// tree directories -> (forest kind, first global tree id) of the engine built from them (Forest<S>::load)
struct ForestDirs {
  ffd_engine* engine = nullptr;
  std::string hp_dir;
  std::vector<std::string> mp_dirs;
  int mp_ntrees = 20;
};
// The live FaceForests' engines, in construction order.  The reference's ImageSample, MeanShift and Forest::load
// signatures carry no engine (src/ImageSample.cpp:11-20, include/MeanShift.hpp:41-76, include/Forest.hpp:103-129),
// so with ONE FaceForest alive they use its engine; with several alive a call that names no engine is ambiguous and
// fails (default_engine) instead of binding to whichever was constructed last.
struct Registry {
  std::mutex mu;
  std::vector<ForestDirs> live;
};
inline Registry& registry() {
  static Registry r;
  return r;
}
inline void register_engine(const ForestDirs& d) {
  std::lock_guard<std::mutex> g(registry().mu);
  registry().live.push_back(d);
}
inline void unregister_engine(ffd_engine* e) {
  std::lock_guard<std::mutex> g(registry().mu);
  auto& v = registry().live;
  for (size_t i = 0; i < v.size(); i++)
    if (v[i].engine == e) {
      v.erase(v.begin() + (std::ptrdiff_t)i);
      break;
    }
}
inline size_t live_engines() {
  std::lock_guard<std::mutex> g(registry().mu);
  return registry().live.size();
}
// The engine a call without one uses: the only live FaceForest's, nullptr when none is alive; throws when more than
// one is alive (`who` names the call in the message).
inline ffd_engine* default_engine(const char* who) {
  std::lock_guard<std::mutex> g(registry().mu);
  const auto& v = registry().live;
  if (v.size() > 1)
    throw std::runtime_error(std::string(who) + ": " + std::to_string(v.size()) +
                             " FaceForests are alive, so the engine is ambiguous; pass one explicitly");
  return v.empty() ? nullptr : v[0].engine;
}
// Calls into an engine one at a time, with the error text read under the same lock.  The C ABI takes one
// caller per engine at a time (ffd.h), while the reference's callers evaluate forests and samples from pool
// threads (face_utils.cpp:210-216, 267-274) and distinct Forest / ImageSample objects share their engine.
// Lock order: a Forest's cache or an ImageSample's state first, then the engine.
inline std::mutex& engine_mutex(const ffd_engine* e) {
  static std::mutex mu;
  static std::unordered_map<const ffd_engine*, std::unique_ptr<std::mutex>> m;
  std::lock_guard<std::mutex> g(mu);
  std::unique_ptr<std::mutex>& p = m[e];
  if (!p) p.reset(new std::mutex());
  return *p;
}
template <class F>
ffd_status engine_call(ffd_engine* e, std::string& err, F f) {
  std::lock_guard<std::mutex> g(engine_mutex(e));
  const ffd_status st = f();
  if (st != FFD_OK) err = ffd_last_error(e);
  return st;
}
inline uint64_t next_sample_id() {
  static std::atomic<uint64_t> n{0};
  return ++n;
}
inline std::string model_cache_path(const std::string& key) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a of the inputs (paths, sizes, modification times)
  for (unsigned char c : key) h = (h ^ c) * 1099511628211ull;
  const char* dir = std::getenv("FFD_MODEL_CACHE");
  std::string d = dir ? dir : "";
  if (d.empty()) {
    const char* xdg = std::getenv("XDG_CACHE_HOME");
    const char* home = std::getenv("HOME");
    d = xdg ? std::string(xdg) + "/ffd" : home ? std::string(home) + "/.cache/ffd"
                                              : "/tmp/ffd-" + std::to_string((long)getuid());  // (per user)
  }
  std::string p;
  for (size_t i = 1; i <= d.size(); i++)  // mkdir -p
    if (i == d.size() || d[i] == '/') (void)mkdir(d.substr(0, i).c_str(), 0700);
  char name[64];
  std::snprintf(name, sizeof name, "/ffd_model_%016llx.bin", (unsigned long long)h);
  return d + name;
}
// a converted model in the cache is used only if it is a complete FFDMODEL container (its directory of arrays
// ends inside the file): a file left by a crashed or concurrent writer is converted again
inline bool model_file_ok(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  char head[16];
  if (!f.read(head, 16) || std::string(head, 8) != "FFDMODEL") return false;
  uint32_t ver, n;
  std::memcpy(&ver, head + 8, 4);
  std::memcpy(&n, head + 12, 4);
  if (ver != 1 || n == 0 || n > 4096) return false;
  uint64_t end = 0;
  for (uint32_t i = 0; i < n; i++) {  // entries (ffd_model_format.h): name[48] dtype[8] ndim pad shape[4] offset nbytes
    char e[112];
    if (!f.read(e, 112)) return false;
    uint64_t off, nb;
    std::memcpy(&off, e + 96, 8);
    std::memcpy(&nb, e + 104, 8);
    end = std::max(end, off + nb);
  }
  f.seekg(0, std::ios::end);
  return (uint64_t)f.tellg() >= end;
}
inline std::string file_key(const std::string& p) {
  struct stat st;
  if (stat(p.c_str(), &st) != 0) return p + "|missing";
  return p + "|" + std::to_string((long long)st.st_size) + "|" + std::to_string((long long)st.st_mtime);
}
inline ffd_forest_param to_c(const ForestParam& p) {
  ffd_forest_param c;
  c.max_depth = p.max_depth; c.min_patches = p.min_patches; c.ntests = p.ntests; c.ntrees = p.ntrees;
  c.nimages = p.nimages; c.npatches = p.npatches; c.face_size = p.face_size;
  c.patch_size_ratio = p.patch_size_ratio;
  c.tree_path = p.tree_path.c_str();
  c.image_path = p.image_path.c_str();
  c.features = reinterpret_cast<const int32_t*>(p.features.data());
  c.n_features = (int32_t)p.features.size();
  return c;
}
inline std::vector<std::string> subdirs(const std::string& dir) {
  int64_t n = 0;
  std::vector<std::string> out;
  if (ffd_forest_subdirs(dir.c_str(), nullptr, 0, &n) != FFD_OK) return out;
  std::string buf((size_t)n, '\0');
  if (ffd_forest_subdirs(dir.c_str(), &buf[0], n, &n) != FFD_OK) return out;
  for (size_t b = 0; b < buf.size();) {
    const size_t e = buf.find('\0', b);
    out.push_back(buf.substr(b, e - b));
    b = e + 1;
  }
  return out;
}
inline float cv_round_f(float v) { return std::nearbyint(v); }  // cvRound: round half to even
}  // namespace detail

#ifndef FFD_HAVE_OPENCV
// cv::CascadeClassifier stand-in, the classifier the static FaceForest::detectFace takes (include/FaceForest.hpp:
// 125-132): load() reads the XML (OpenCV's BOOST / HAAR stump format) into an engine of its own that holds only
// that cascade on the GPU (ffd_detector_create, device $FFD_DEVICE or 0); detectFace runs it.  false (and
// empty()) when the file cannot be read, as OpenCV's load.  Copies share the detector.
class CascadeClassifier {
 public:
  CascadeClassifier() = default;
  explicit CascadeClassifier(const std::string& filename) { load(filename); }
  bool load(const std::string& filename) {
    det_.reset();
    path_.clear();
    const char* dv = std::getenv("FFD_DEVICE");
    ffd_engine* e = nullptr;
    if (ffd_detector_create(filename.c_str(), dv ? std::atoi(dv) : 0, &e) != FFD_OK) {
      err_ = ffd_last_error(nullptr);
      return false;
    }
    det_ = std::shared_ptr<ffd_engine>(e, [](ffd_engine* x) {
      std::lock_guard<std::mutex> g(detail::engine_mutex(x));
      ffd_engine_destroy(x);
    });
    path_ = filename;
    return true;
  }
  bool empty() const { return !det_; }
  const std::string& path() const { return path_; }
  const std::string& last_error() const { return err_; }
  ffd_engine* engine() const { return det_.get(); }

 private:
  std::string path_, err_;
  std::shared_ptr<ffd_engine> det_;
};
#endif

// ------------------------------------------------------------------ ImageSample --
// ImageSample (include/ImageSample.hpp:146-190, src/ImageSample.cpp:11-20,77-90): the 38 integral feature
// channels of a scaled gray face, extracted by the engine's HIP kernels and kept in HBM (ffd_sample_create).
// features must be {0, 1, 2} (the configuration of the pretrained forests, data/config_ffd.txt); use_integral
// selects how the reference evaluates a test (integral image or pixel sums), which gives the same value, so
// both are accepted.
class ImageSample {
 public:
  ImageSample(const Mat img, std::vector<int> features, bool use_integral = false, ffd_engine* engine = nullptr)
      : ImageSample(mat_data(img), img.cols, img.rows, (size_t)mat_step(img), features, use_integral, engine) {
    if (img.channels() != 1) throw std::invalid_argument("ImageSample: the image must be 8-bit single-channel (gray)");
  }
  ImageSample(const uint8_t* gray, int cols, int rows, size_t step, const std::vector<int>& features = {0, 1, 2},
              bool useIntegral = true, ffd_engine* engine = nullptr)
      : st_(std::make_shared<State>()) {
    (void)useIntegral;
    std::vector<int> f(features);
    std::sort(f.begin(), f.end());
    if (f != std::vector<int>({0, 1, 2}))
      throw std::invalid_argument("ImageSample: only features {0,1,2} are supported (the pretrained forests' channels)");
    st_->w = cols;
    st_->hgt = rows;
    st_->id = detail::next_sample_id();
    st_->gray.resize((size_t)cols * rows);  // (the training images of Tree<MPSample>(samples, ...))
    for (int y = 0; y < rows; y++) std::memcpy(&st_->gray[(size_t)y * cols], gray + (size_t)y * step, (size_t)cols);
    // the channels on the device now, as the reference's constructor computes them; without an engine (a training
    // program that builds ImageSamples before any FaceForest, demo.cpp:86-96) on first use, with the engine current then
    st_->engine = engine ? engine : detail::default_engine("ImageSample");
    if (st_->engine) st_->create();
  }
  // the 8-bit gray image the channels were extracted from (rows x cols, row pitch cols)
  const std::vector<uint8_t>& gray() const { return st_->gray; }
  int width() const { return st_->w; }
  int height() const { return st_->hgt; }
  ffd_engine* engine() const { return ensure()->engine; }
  ffd_sample* handle() const { return ensure()->h; }
  uint64_t id() const { return st_->id; }
  // the channels as 38 u32 integral planes [38][rows+1][cols+1] (downloaded on first use)
  const uint32_t* channels() const {
    ensure();
    std::lock_guard<std::mutex> g(st_->mu);
    if (st_->ch.empty()) {
      st_->ch.resize((size_t)38 * (st_->hgt + 1) * (st_->w + 1));
      std::string err;
      if (detail::engine_call(st_->engine, err, [&] { return ffd_sample_channels(st_->h, st_->ch.data()); }) != FFD_OK) {
        st_->ch.clear();
        throw std::runtime_error("ImageSample: " + err);
      }
    }
    return st_->ch.data();
  }

 private:
  struct State {
    ffd_engine* engine = nullptr;
    ffd_sample* h = nullptr;
    int w = 0, hgt = 0;
    uint64_t id = 0;
    std::mutex mu;
    std::vector<uint32_t> ch;
    std::vector<uint8_t> gray;
    void create() {
      std::string err;
      if (detail::engine_call(engine, err, [&] { return ffd_sample_create(engine, gray.data(), w, hgt, (int32_t)w, &h); }) != FFD_OK)
        throw std::runtime_error("ImageSample: " + err);
    }
    ~State() {
      if (!h) return;
      std::lock_guard<std::mutex> g(detail::engine_mutex(engine));
      ffd_sample_destroy(h);
    }
  };
  std::shared_ptr<State> st_;  // copies share the device sample (the reference copies cv::Mat headers)
  State* ensure() const {
    std::lock_guard<std::mutex> g(st_->mu);
    if (!st_->h) {
      if (!st_->engine) st_->engine = detail::default_engine("ImageSample");
      if (!st_->engine) throw std::runtime_error("ImageSample: no FaceForest engine");
      st_->create();
    }
    return st_.get();
  }
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
  static constexpr int default_step = 4;  // HeadPoseEstimatorOption::step_size
  const ImageSample* image;
  Rect roi;
  HeadPoseSample(const ImageSample* i, Rect r) : image(i), roi(r) {}
  Rect getPatch() const { return roi; }
};
struct MPSample {
  typedef MPLeaf Leaf;
  static constexpr int default_step = 3;  // MultiPartEstimatorOption::step_size
  const ImageSample* image;
  Rect roi;
  MPSample(const ImageSample* i, Rect r) : image(i), roi(r) {}
  // Training (MPSample.hpp:36-44, MPSample.cpp:13-41): the annotated landmarks of the sample's image; the part
  // offsets and probabilities are computed where the tree is grown (Tree<MPSample>(samples, ...), on the GPU)
  MPSample(const ImageSample* i, Rect r, const std::vector<Point> annotation_parts, float face_size_, bool label_,
           float lamda_ = 0.125f)
      : image(i), roi(r), parts(annotation_parts), face_size(face_size_), label(label_), lamda(lamda_) {}
  Rect getPatch() const { return roi; }
  std::vector<Point> parts;  // (training samples only)
  float face_size = 0.f;
  bool label = false;
  float lamda = 0.125f;
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

// Tree<S> (include/Tree.hpp): a tree of the engine's model, by global id (head pose 0..14, FFD forest*20 + t), or
// a tree grown from training samples.
template <class S> struct Tree {
  int32_t id = -1;
  ffd_engine* engine = nullptr;
  Tree() = default;
  Tree(int32_t id_, ffd_engine* e) : id(id_), engine(e) {}
  // Training (Tree.hpp:43-64: grow from the samples, then save() to save_path), S = MPSample: the samples' images
  // and patches go to the GPU trainer (ffd_train_mp_tree_patches); the rng's type is the caller's (the reference
  // passes a boost::mt19937*; its draws were spent on the patches, the split search has generators of its own,
  // seeded per stripe by std::time as SplitGen does, or by $FFD_SPLIT_SEED).  Throws on failure.
  template <class Rng>
  Tree(const std::vector<S*>& samples, ForestParam param, Rng* rng, std::string save_path) {
    (void)rng;
    std::vector<const ImageSample*> imgs;
    std::vector<std::vector<int32_t>> parts;
    std::vector<int32_t> patches;
    for (const S* smp : samples) {
      size_t k = 0;
      while (k < imgs.size() && imgs[k] != smp->image) k++;
      std::vector<int32_t> pv;
      for (const Point& q : smp->parts) pv.insert(pv.end(), {q.x, q.y});
      if (pv.size() != 2 * FFD_NUM_LANDMARKS) throw std::invalid_argument("Tree: a training sample needs 10 parts");
      if (smp->lamda != 0.125f || (int)smp->face_size != param.face_size)
        throw std::invalid_argument("Tree: training samples must use lamda 0.125 and the param's face_size");
      if (k == imgs.size()) {
        imgs.push_back(smp->image);
        parts.push_back(pv);
      } else if (parts[k] != pv) {
        throw std::invalid_argument("Tree: the samples of one image must carry the same annotation");
      }
      patches.insert(patches.end(), {(int32_t)k, smp->roi.x, smp->roi.y});
    }
    std::vector<ffd_train_image> ti(imgs.size());
    for (size_t k = 0; k < imgs.size(); k++)
      ti[k] = ffd_train_image{imgs[k]->gray().data(), imgs[k]->width(), imgs[k]->height(), imgs[k]->width(),
                              parts[k].data()};
    ffd_train_param tp;
    ffd_train_param_init(&tp);
    tp.max_depth = param.max_depth; tp.min_patches = param.min_patches; tp.ntests = param.ntests;
    tp.ntrees = param.ntrees; tp.nimages = param.nimages; tp.npatches = param.npatches;
    tp.face_size = param.face_size; tp.patch_size_ratio = param.patch_size_ratio;
    tp.tree_path = param.tree_path.c_str();
    tp.image_path = param.image_path.c_str();
    tp.save_path = save_path.c_str();
    const char* seed = std::getenv("FFD_SPLIT_SEED");
    tp.split_seed = seed ? (uint32_t)std::strtoul(seed, nullptr, 10) : (uint32_t)std::time(nullptr);
    const char* dv = std::getenv("FFD_DEVICE");
    tp.device = dv ? std::atoi(dv) : 0;
    ffd_trained_tree* t = nullptr;
    if (ffd_train_mp_tree_patches(&tp, ti.data(), (int32_t)ti.size(), patches.data(), (int64_t)(patches.size() / 3), &t) != FFD_OK)
      throw std::runtime_error(std::string("Tree: training failed: ") + ffd_train_last_error());
    trained.reset(t, ffd_trained_tree_free);
    if (ffd_trained_tree_save(t, save_path.c_str()) != FFD_OK)  // Tree::save (Tree.hpp:239-256)
      throw std::runtime_error(std::string("Tree: cannot save ") + save_path + ": " + ffd_train_last_error());
  }
  std::shared_ptr<ffd_trained_tree> trained;  // (a grown tree: ffd_trained_tree_* reads its nodes and leaves)
};

// Forest<S> (include/Forest.hpp): a list of the engine's trees (value semantics, as the reference's vector of
// Tree*).  Copies share the leaf payloads and the per-sample evaluation cache (the reference binds the Forest
// BY VALUE into every pool task, face_utils.cpp:215,273), so the Leaf* of evaluateMT stay valid while any copy
// lives and every task's copy reads the one grid evaluation.
template <class S> class Forest {
 public:
  typedef typename S::Leaf Leaf;
  Forest() : sh_(std::make_shared<Shared>()) {}
  Forest(ffd_engine* e, std::vector<int32_t> trees) : sh_(std::make_shared<Shared>()) {
    engine_ = e;
    for (int32_t t : trees) addTree(t);
  }
  int numberOfTrees() const { return (int)sh_->list->ids.size(); }
  const std::vector<int32_t>& treeIds() const { return sh_->list->ids; }
  ffd_engine* engine() const { return engine_; }
  void setParam(ForestParam fp) { mut_shared().param = std::make_shared<const ForestParam>(std::move(fp)); }
  ForestParam getParam() const { return sh_->param ? *sh_->param : ForestParam(); }
  // Forest::addTree / getTree / cleanForest (Forest.hpp:41-68), as FaceForest::analyzeFace composes the
  // per-face forest from the jungle (FaceForest.cpp:239-250)
  void addTree(Tree<S>* tree) {
    if (!engine_) engine_ = tree->engine;
    addTree(tree->id);
  }
  void addTree(int32_t id) {
    TreeList& l = mut();
    l.ids.push_back(id);
    l.trees.push_back(Tree<S>(id, engine_));
  }
  Tree<S>* getTree(int idx) { return &mut().trees.at(idx); }
  void cleanForest() { mut_shared().list = std::make_shared<TreeList>(); }
  // the patch grid step of the speculative evaluation (0: S::default_step)
  void setGridStep(int step) { grid_step_ = step; }

  // Forest<S>::load(path, ForestParam, max_trees) (Forest.hpp:103-129): the forest of the current engine that
  // was converted from the tree directory `path` (FaceForest(FaceForestOptions) records them), its first trees
  // as the reference's loop admits them.  false (with an ERROR line on stderr, as Forest::load_tree) when no
  // engine holds that directory.
  bool load(std::string path, ForestParam fp, int max_trees = -1) { return load(path, fp, max_trees, nullptr); }
  // ... from the trees of a given engine (nullptr: the live FaceForest whose options name the directory; with
  // several such FaceForests alive the call fails instead of picking one)
  bool load(std::string path, ForestParam fp, int max_trees, ffd_engine* engine) {
    setParam(fp);
    if (max_trees == -1) max_trees = fp.ntrees;
    auto same = [](const std::string& a, const std::string& b) {
      char ra[4096], rb[4096];
      return a == b || (realpath(a.c_str(), ra) && realpath(b.c_str(), rb) && std::string(ra) == std::string(rb));
    };
    int base = -1, holders = 0;
    ffd_engine* eng = nullptr;
    {
      std::lock_guard<std::mutex> g(detail::registry().mu);
      for (const detail::ForestDirs& d : detail::registry().live) {
        if (engine && d.engine != engine) continue;
        int b = -1;
        if (ForestKind<S>::value == FFD_FOREST_HEADPOSE && !d.hp_dir.empty() && same(path, d.hp_dir)) b = 0;
        if (ForestKind<S>::value == FFD_FOREST_FFD)
          for (size_t i = 0; i < d.mp_dirs.size(); i++)
            if (same(path, d.mp_dirs[i])) b = (int)i * d.mp_ntrees;
        if (b >= 0) {
          holders++;
          base = b;
          eng = d.engine;
        }
      }
    }
    if (holders > 1) {
      std::fprintf(stderr, "ERROR: Forest::load: %d FaceForests hold the trees of %s; pass the engine\n", holders,
                   path.c_str());
      return false;
    }
    if (base < 0 || !eng) {
      std::fprintf(stderr, "ERROR: Forest::load: no engine holds the trees of %s\n", path.c_str());
      return false;
    }
    engine_ = eng;
    for (int i = 0; i < fp.ntrees; i++) {
      if (numberOfTrees() > max_trees) continue;
      addTree(base + i);
    }
    return true;
  }

  // Forest<S>::evaluateMT(const S*, S::Leaf**) (Forest.hpp:80-90): leafs[t] = the leaf tree t reaches.
  // A patch of the grid this thread read last is served from the thread's reference to that (immutable) grid,
  // with no lock; any other call goes through the cache under its mutex.
  void evaluateMT(const S* sample, Leaf** leafs) const {
    const Grid* g = local_grid(sample);
    const size_t row = g ? g->row_of(sample->roi.x, sample->roi.y) : npos;
    if (row != npos) {  // Leaf* = the tree's array + (ordinal - its first ordinal), one offset per tree
      const int32_t* id = &g->ids[row];
      const intptr_t* off = g->off.data();
      for (size_t t = 0; t < g->T; t++) leafs[t] = reinterpret_cast<Leaf*>(off[t] + (intptr_t)id[t] * (intptr_t)sizeof(Leaf));
      return;
    }
    const std::vector<int32_t>& trees = sh_->list->ids;
    std::vector<int32_t> ids(trees.size());
    std::lock_guard<std::mutex> lk(sh_->cache->mu);
    eval_one(sample, ids.data());
    for (size_t t = 0; t < trees.size(); t++) leafs[t] = leaf_of_tree(trees[t], ids[t]);
  }
  // the same with the model's leaf ordinals (ffd_forest_leaves gives their payloads)
  void evaluateMT(const S* sample, int32_t* leafs) const {
    const Grid* g = local_grid(sample);
    const size_t row = g ? g->row_of(sample->roi.x, sample->roi.y) : npos;
    if (row != npos) {
      std::copy(&g->ids[row], &g->ids[row] + g->T, leafs);
      return;
    }
    std::lock_guard<std::mutex> lk(sh_->cache->mu);
    eval_one(sample, leafs);
  }
  // the payload of a leaf ordinal (the reference: TreeNode::getLeaf, TreeNode.hpp:61-66)
  Leaf& leaf(int32_t ordinal) const {
    std::lock_guard<std::mutex> g(sh_->cache->mu);
    return *leaf_locked(ordinal);
  }

 private:
  static constexpr size_t npos = ~(size_t)0;
  struct Grid;
  struct Cache {
    std::mutex mu;
    // leaf payloads tree by tree: a tree's leaves are filled together the first time one of them is asked for
    // (the reference holds every loaded tree's leaves in memory, Forest::load), in one array per tree, so a
    // Leaf* is the tree's array + arithmetic and stays valid while the cache lives
    std::vector<std::unique_ptr<Leaf[]>> arr;  // by tree id
    std::vector<int32_t> first, count;         // by tree id: leaf ordinals [first, first + count); count -1: unknown
    std::shared_ptr<Grid> grid;  // the last (sample, tree list) evaluated
  };
  // the speculative grid evaluation of one (sample, tree list): patches (x0 + i step, y0 + j step).  Never changed
  // once published, so a thread holding a reference reads it without the cache's lock.
  struct Grid {
    uint64_t sample = 0;
    std::vector<int32_t> trees;  // the tree list it was evaluated for
    size_t T = 0;
    int ny = 0;
    std::vector<int32_t> col, row;  // patch x / y -> grid index i / j (-1: off the grid)
    std::vector<int32_t> ids;       // leaf ordinals [(i * ny + j) * T + t]
    std::vector<intptr_t> off;      // per tree: its leaf array's address - its first ordinal * sizeof(Leaf)
    size_t row_of(int x, int y) const {  // by table, no divisions per call
      const int i = (unsigned)x < col.size() ? col[x] : -1, j = (unsigned)y < row.size() ? row[y] : -1;
      return i < 0 || j < 0 ? npos : ((size_t)i * ny + j) * T;
    }
  };
  // a thread's last grid: the cache it belongs to (kept alive: the grid's Leaf* point into it), the sample and the
  // TreeList uid it was validated for
  struct Local {
    std::shared_ptr<Cache> cache;
    uint64_t sample = 0, list_uid = 0;
    std::shared_ptr<const Grid> grid;
  };
  static Local& local() {
    static thread_local Local l;
    return l;
  }
  // the tree list, shared by copies until one of them changes it (a copy per evaluateMT call, as the reference
  // binds the forest by value into every task, then costs a reference count, not a list copy)
  struct TreeList {
    std::vector<int32_t> ids;
    std::deque<Tree<S>> trees;
    uint64_t uid = detail::next_sample_id();  // a new one with every change (the cache's key)
  };
  // what copies share: the tree list, the param and the evaluation cache behind ONE reference count, so the copy
  // per evaluateMT call costs one atomic increment (copy-on-write: a copy that changes its list or param gets its
  // own Shared, still over the same cache, which is keyed by the tree list)
  struct Shared {
    std::shared_ptr<TreeList> list = std::make_shared<TreeList>();
    std::shared_ptr<const ForestParam> param;
    std::shared_ptr<Cache> cache = std::make_shared<Cache>();
  };
  ffd_engine* engine_ = nullptr;
  int grid_step_ = 0;
  std::shared_ptr<Shared> sh_;
  Shared& mut_shared() {
    if (sh_.use_count() > 1) sh_ = std::make_shared<Shared>(*sh_);
    return *sh_;
  }
  TreeList& mut() {
    Shared& x = mut_shared();
    if (x.list.use_count() > 1) x.list = std::make_shared<TreeList>(*x.list);
    x.list->uid = detail::next_sample_id();
    return *x.list;
  }

  // an engine call under the engine's lock (detail::engine_call); a failure throws with its error text
  template <class F> void call(ffd_engine* e, F f) const {
    std::string err;
    if (detail::engine_call(e, err, f) != FFD_OK) throw std::invalid_argument(err);
  }
  // tree t's leaf ordinal range (cached); false for a tree id the engine does not have
  bool tree_range(int32_t t, int32_t& first, int32_t& count) const {
    Cache& c = *sh_->cache;
    if (t < 0) return false;
    if ((size_t)t >= c.count.size()) {
      c.first.resize((size_t)t + 1, 0);
      c.count.resize((size_t)t + 1, -1);
      c.arr.resize((size_t)t + 1);
    }
    if (c.count[t] < 0) {
      std::string err;
      if (detail::engine_call(engine_, err, [&] {
            return ffd_forest_tree_leaves(engine_, ForestKind<S>::value, t, &c.first[t], &c.count[t]);
          }) != FFD_OK) {
        c.count[t] = -1;
        return false;
      }
    }
    first = c.first[t];
    count = c.count[t];
    return true;
  }
  // tree t's leaf array, filled on first use
  Leaf* tree_leaves(int32_t t) const {
    Cache& c = *sh_->cache;
    int32_t first = 0, count = 0;
    if (!tree_range(t, first, count)) throw std::invalid_argument("Forest: no tree " + std::to_string(t));
    if (!c.arr[t]) {
      std::vector<int32_t> ord((size_t)count);
      for (int32_t i = 0; i < count; i++) ord[i] = first + i;
      std::vector<typename ForestKind<S>::Raw> raw((size_t)count);
      if (count) call(engine_, [&] { return ffd_forest_leaves(engine_, ForestKind<S>::value, ord.data(), count, raw.data()); });
      std::unique_ptr<Leaf[]> a(new Leaf[(size_t)std::max(count, 1)]);
      for (int32_t i = 0; i < count; i++) ForestKind<S>::fill(raw[i], a[i]);
      c.arr[t] = std::move(a);
    }
    return c.arr[t].get();
  }
  Leaf* leaf_of_tree(int32_t t, int32_t ordinal) const {
    Leaf* a = tree_leaves(t);
    return a + (ordinal - sh_->cache->first[t]);
  }
  // the payload of any leaf ordinal: the tree holding it among this forest's trees, else among the engine's
  Leaf* leaf_locked(int32_t ordinal) const {
    int32_t first = 0, count = 0;
    for (int32_t t : sh_->list->ids)
      if (tree_range(t, first, count) && ordinal >= first && ordinal - first < count) return leaf_of_tree(t, ordinal);
    for (int32_t t = 0; tree_range(t, first, count); t++)
      if (ordinal >= first && ordinal - first < count) return leaf_of_tree(t, ordinal);
    typename ForestKind<S>::Raw raw;  // (no tree holds it: the engine's error for a bad ordinal)
    call(engine_, [&] { return ffd_forest_leaves(engine_, ForestKind<S>::value, &ordinal, 1, &raw); });
    throw std::invalid_argument("Forest: no leaf " + std::to_string(ordinal));
  }
  void eval_one(const S* sample, int32_t* ids) const {
    const int32_t xy[2] = {sample->roi.x, sample->roi.y};
    call(sample->image->engine(), [&] {
      return ffd_sample_eval_leaves(sample->image->handle(), ForestKind<S>::value, xy, 1, sh_->list->ids.data(),
                                    (int32_t)sh_->list->ids.size(), ids);
    });
  }
  // The grid of (sample, this tree list), evaluated first when the cache holds another sample or tree list; null
  // when the patch's grid cannot be made (a patch outside the image or no trees: evaluated alone).
  const Grid* local_grid(const S* sample) const {
    Local& l = local();
    const ImageSample& im = *sample->image;
    const TreeList& L = *sh_->list;
    if (l.grid && l.cache == sh_->cache && l.sample == im.id() && l.list_uid == L.uid) return l.grid.get();
    Cache& c = *sh_->cache;
    std::lock_guard<std::mutex> lk(c.mu);
    const std::vector<int32_t>& ids = L.ids;
    const int x = sample->roi.x, y = sample->roi.y, P = 31, T = (int)ids.size();
    if (!c.grid || c.grid->sample != im.id() || c.grid->trees != ids) {
      if (x < 0 || y < 0 || x + P > im.width() || y + P > im.height() || T == 0) return nullptr;
      const int step = grid_step_ > 0 ? grid_step_ : S::default_step;
      // the grid being replaced is rebuilt in place when no thread holds it any more (its storage is warm)
      if (l.grid == c.grid) l.grid.reset();
      std::shared_ptr<Grid> g = c.grid && c.grid.use_count() == 1 ? std::move(c.grid) : std::make_shared<Grid>();
      g->sample = im.id();
      g->trees = ids;
      g->T = (size_t)T;
      const int x0 = x % step, y0 = y % step, nx = (im.width() - P - x0) / step + 1;
      g->ny = (im.height() - P - y0) / step + 1;
      g->col.assign((size_t)im.width(), -1);
      g->row.assign((size_t)im.height(), -1);
      for (int k = 0; k < nx; k++) g->col[(size_t)(x0 + k * step)] = k;
      for (int k = 0; k < g->ny; k++) g->row[(size_t)(y0 + k * step)] = k;
      g->ids.resize((size_t)nx * g->ny * T);
      call(im.engine(), [&] {
        return ffd_sample_eval_grid(im.handle(), ForestKind<S>::value, x0, y0, step, nx, g->ny, ids.data(), T,
                                    g->ids.data());
      });
      // every leaf payload of the list's trees, the first time a tree is used; a grid leaf's Leaf* is then its
      // tree's array + (ordinal - the tree's first ordinal), computed per call (no pointer table to write)
      g->off.resize((size_t)T);
      for (int t = 0; t < T; t++)
        g->off[t] = (intptr_t)tree_leaves(ids[t]) - (intptr_t)c.first[ids[t]] * (intptr_t)sizeof(Leaf);
      c.grid = std::move(g);
    }
    l.cache = sh_->cache;
    l.sample = im.id();
    l.list_uid = L.uid;
    l.grid = c.grid;
    return l.grid.get();
  }
};

// ------------------------------------------------------------------ MeanShift --
// MeanShift::shift (include/MeanShift.hpp:41-76) on the GPU (ffd_meanshift) with the current engine.
class MeanShift {
 public:
  static void shift(const std::vector<Vote>& votes, Point& result, MeanShiftOption& option) {
    shift(votes, result, option.max_iterations, option.kernel_size, option.stopping_criteria);
  }
  static void shift(const std::vector<Vote>& votes, Point& result, int num_iterations, int kernel,
                    float stopping_criteria) {
    float m[2];
    mode(votes, m, num_iterations, kernel, stopping_criteria);
    result = Point((int)detail::cv_round_f(m[0]), (int)detail::cv_round_f(m[1]));  // Point_<float> -> Point_<int>
  }
  // the mode before rounding
  static void mode(const std::vector<Vote>& votes, float* mean_xy, int num_iterations = 7, int kernel = 10,
                   float stopping_criteria = 0.05f) {
    mode(votes, mean_xy, num_iterations, kernel, stopping_criteria, detail::default_engine("MeanShift"));
  }
  // the same on a given engine (FaceForest::engine()), for a program with several FaceForests alive
  static void shift(const std::vector<Vote>& votes, Point& result, int num_iterations, int kernel,
                    float stopping_criteria, ffd_engine* e) {
    float m[2];
    mode(votes, m, num_iterations, kernel, stopping_criteria, e);
    result = Point((int)detail::cv_round_f(m[0]), (int)detail::cv_round_f(m[1]));
  }
  static void mode(const std::vector<Vote>& votes, float* mean_xy, int num_iterations, int kernel,
                   float stopping_criteria, ffd_engine* e) {
    if (!e) throw std::runtime_error("MeanShift: no FaceForest engine");
    std::vector<ffd_vote> v(votes.size());
    for (size_t i = 0; i < votes.size(); i++)
      v[i] = ffd_vote{votes[i].pos.x, votes[i].pos.y, votes[i].weight, votes[i].check ? 1 : 0};
    const ffd_meanshift_option o{kernel, num_iterations, stopping_criteria};
    std::string err;
    if (detail::engine_call(e, err, [&] { return ffd_meanshift(e, v.data(), (int32_t)v.size(), &o, mean_xy); }) != FFD_OK)
      throw std::runtime_error("MeanShift: " + err);
  }
};

// ------------------------------------------------------------------ face_utils --
// getHeadPoseVotesMT (face_utils.cpp:183-242) over any head-pose forest: the patch grid of face_bbox, every tree's
// leaf through Forest::evaluateMT (one GPU evaluation of the grid), then the reference's float sums on the host.
inline void getHeadPoseVotesMT(const ImageSample& sample, const Forest<HeadPoseSample>& forest, Rect face_bbox,
                               float* headpose, float* variance,
                               HeadPoseEstimatorOption options = HeadPoseEstimatorOption()) {
  const int patch_size = forest.getParam().getPatchSize() > 0 ? forest.getParam().getPatchSize() : 31;
  const int num_trees = forest.numberOfTrees();
  std::vector<HeadPoseSample> samples;
  for (int x = face_bbox.x; x < face_bbox.x + face_bbox.width - patch_size; x += options.step_size)
    for (int y = face_bbox.y; y < face_bbox.y + face_bbox.height - patch_size; y += options.step_size)
      samples.push_back(HeadPoseSample(&sample, Rect(x, y, patch_size, patch_size)));
  Forest<HeadPoseSample> f(forest);
  f.setGridStep(options.step_size);
  std::vector<HeadPoseLeaf*> leafs(samples.size() * num_trees);
  for (size_t i = 0; i < samples.size(); i++) f.evaluateMT(&samples[i], &leafs[i * num_trees]);
  float n = 0, sum = 0, sum_sq = 0;
  for (size_t i = 0; i < leafs.size(); ++i) {
    if (leafs[i]->hp_foreground > options.min_foreground_probability) {
      float m = 0;  // predicted label [0..4]
      for (int j = 0; j < options.num_head_pose_labels; j++) m += leafs[i]->hp_labels[j] * j;
      m /= (leafs[i]->hp_nsamples * leafs[i]->hp_foreground);
      sum += m;
      sum_sq += m * m;
      n++;
    }
  }
  float mean = sum / n;
  float var = (sum_sq / n) - (mean * mean);
  mean -= 2;
  var *= NORM_HEADPOSE_VARIANCE_FACTOR;
  *headpose = mean;
  *variance = var;
}

// getFacialFeaturesVotesMT (face_utils.cpp:244-302): votes[i] (the caller sizes votes to the parts) gains one
// vote per (patch, tree) leaf that passes the option's filter, in the reference's patch-major, tree-minor order.
inline void getFacialFeaturesVotesMT(const ImageSample& sample, const Forest<MPSample>& forest, Rect face_bbox,
                                     std::vector<std::vector<Vote>>& votes,
                                     MultiPartEstimatorOption options = MultiPartEstimatorOption()) {
  const int patch_size = forest.getParam().getPatchSize() > 0 ? forest.getParam().getPatchSize() : 31;
  std::vector<MPSample> samples;
  for (int x = face_bbox.x; x < face_bbox.x + face_bbox.width - patch_size; x += options.step_size)
    for (int y = face_bbox.y; y < face_bbox.y + face_bbox.height - patch_size; y += options.step_size)
      samples.push_back(MPSample(&sample, Rect(x, y, patch_size, patch_size)));
  const int num_trees = forest.numberOfTrees();
  Forest<MPSample> f(forest);
  f.setGridStep(options.step_size);
  std::vector<MPLeaf*> leafs(samples.size() * num_trees);
  for (size_t i = 0; i < samples.size(); i++) f.evaluateMT(&samples[i], &leafs[i * num_trees]);
  for (size_t k = 0; k < leafs.size(); k++) {
    const MPLeaf* l = leafs[k];
    const int offset_x = samples[k / num_trees].getPatch().x + patch_size / 2;
    const int offset_y = samples[k / num_trees].getPatch().y + patch_size / 2;
    for (size_t i = 0; i < votes.size(); i++) {
      float min_pf = options.min_pf;
      if (i == 0 || i == 7) min_pf *= 1.5;  // probability in outer eye parts
      if (l->mp_foreground > options.min_forground && l->mp_prob_foreground[i] > min_pf &&
          l->mp_parts_variance[i] < options.max_variance && l->mp_samples > options.min_samples) {
        Vote v;
        v.pos.x = l->mp_parts_offset[i].x + offset_x;
        v.pos.y = l->mp_parts_offset[i].y + offset_y;
        v.weight = l->mp_foreground;
        v.check = true;
        votes[i].push_back(v);
      }
    }
  }
}

// areaUnderCurve (face_utils.cpp:304-323): left Riemann sum of the normal density, step 0.01
inline float areaUnderCurve(float x1, float x2, double mean, double std) {
  double sum = 0;
  const double step = 0.01;
  for (double x = x1; x < x2; x += step) {
    const double t = (x - mean) / std;
    sum += std::exp(-0.5 * (t * t)) * step;
  }
  return (float)(sum * 1.0 / (std * std::sqrt(2 * M_PI)));
}

// ------------------------------------------------------------------ FaceForest --
class FaceForest {
 public:
  FaceForest() = default;
  explicit FaceForest(const FaceForestOptions& option) : options_(option) {
    std::string model = option.model_path;
    if (model.empty() && std::getenv("FFD_MODEL")) model = std::getenv("FFD_MODEL");
    if (model.empty() && !option.hp_forest_param.tree_path.empty() && !convert(model)) return;
    if (model.empty()) {
      err_ = "FaceForestOptions: neither model_path / $FFD_MODEL nor hp_forest_param.tree_path is set";
      return;
    }
    ffd_engine_desc d;
    ffd_engine_desc_init(&d);
    d.model_path = model.c_str();
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
      std::fprintf(stderr, "ERROR: (!) Error loading the forests: %s\n", err_.c_str());
    }
    if (engine_) {
      detail::ForestDirs fd;
      fd.engine = engine_;
      fd.hp_dir = options_.hp_forest_param.tree_path;
      fd.mp_dirs = options_.mp_forest_paths;
      if (options_.mp_forest_param.ntrees > 0) fd.mp_ntrees = options_.mp_forest_param.ntrees;
      detail::register_engine(fd);
    }
    fd_option_ = option.fd_option;
  }
  FaceForest(const FaceForest&) = delete;
  FaceForest& operator=(const FaceForest&) = delete;
  FaceForest(FaceForest&& o) noexcept : engine_(o.engine_), err_(std::move(o.err_)), fd_option_(o.fd_option_) {
    o.engine_ = nullptr;
  }
  virtual ~FaceForest() {
    if (engine_) detail::unregister_engine(engine_);
    ffd_engine_destroy(engine_);
  }

  bool is_initialized() const { return engine_ != nullptr; }
  std::string last_error() const { return engine_ ? ffd_last_error(engine_) : err_; }
  const FaceForestOptions& options() const { return options_; }

  // FaceForest::analyzeFace (FaceForest.cpp:183-258)
  void analyzeFace(const Mat img, Rect face_bbox, Face& face) {
    std::vector<Face> faces;
    analyzeImage(img, std::vector<Rect>{face_bbox}, faces);
    face = faces.at(0);
  }

  // FaceForest::detectFace (FaceForest.cpp:136-159) with this object's fd_option, on the GPU.
  void detectFace(const Mat img, std::vector<Rect>& faces_bboxes) { detect(engine_, img, fd_option_, faces_bboxes); }

  // static FaceForest::detectFace (include/FaceForest.hpp:125-132, FaceForest.cpp:136-159) with the classifier it
  // is given.  With OpenCV: the reference itself (the classifier's detectMultiScale on the CPU, then the widening).
  // Without: the classifier's own detector engine (CascadeClassifier::load above) on the GPU.
  static void detectFace(const Mat& img, CascadeClassifier& face_cascade, FaceDetectionOption fd_option,
                         std::vector<Rect>& faces_bboxes) {
#ifdef FFD_HAVE_OPENCV
    const cv::Size min_feature_size(fd_option.min_feature_size, fd_option.min_feature_size);
    face_cascade.detectMultiScale(img, faces_bboxes, fd_option.search_scale_factor, fd_option.min_neighbors, 0,
                                  min_feature_size);
    for (size_t i = 0; i < faces_bboxes.size(); i++) {  // the boxes are too tight for the estimators
      const int offset_x = (int)(faces_bboxes[i].width * 0.05), offset_y = (int)(faces_bboxes[i].width * 0.15);
      const Rect r1(faces_bboxes[i].x - offset_x, faces_bboxes[i].y, faces_bboxes[i].width + (offset_x * 2),
                    faces_bboxes[i].height + (offset_y * 2));
      faces_bboxes[i] = intersect(r1, Rect(0, 0, img.cols, img.rows));
    }
#else
    if (face_cascade.empty()) throw std::runtime_error("detectFace: the CascadeClassifier is not loaded");
    detect(face_cascade.engine(), img, fd_option, faces_bboxes);
#endif
  }

  // FaceForest::analyzeImage (FaceForest.cpp:161-181): detectFace, then analyzeFace on every box (one
  // GPU batch).  Appends to `faces` like the reference.
  void analyzeImage(const Mat img, std::vector<Face>& faces) {
    if (!engine_) throw std::runtime_error("FaceForest not initialised: " + err_);
    ffd_image im{mat_data(img), img.cols, img.rows, mat_step(img)};
    const ffd_detect_options o = detect_options(fd_option_);
    std::vector<ffd_face> out(64);
    int32_t n = 0;
    for (int pass = 0; pass < 2; pass++) {
      std::string err;
      if (detail::engine_call(engine_, err, [&] {
            return ffd_analyze_images(engine_, &im, 1, &o, out.data(), nullptr, (int32_t)out.size(), &n);
          }) != FFD_OK)
        throw std::runtime_error(err);
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
    std::string err;
    const ffd_status st = detail::engine_call(engine_, err, [&] {
      return ffd_analyze_faces(engine_, &im, 1, r.data(), which.data(), (int32_t)r.size(), out.data());
    });
    if (st == FFD_ERR_INVALID_ARGUMENT) throw std::invalid_argument(err);
    if (st != FFD_OK) throw std::runtime_error(err);
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
    std::string err;
    const ffd_status st = detail::engine_call(engine_, err, [&] {
      return ffd_analyze_faces(engine_, im.data(), (int32_t)im.size(), r.data(), nullptr, (int32_t)r.size(), out_.data());
    });
    if (st == FFD_ERR_INVALID_ARGUMENT) throw std::invalid_argument(err);
    if (st != FFD_OK) throw std::runtime_error(err);
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
    Forest<HeadPoseSample> f(engine_, t);
    f.setParam(forest_param(15));
    return f;
  }
  Forest<MPSample> ffdForest(int pose_bin) const {
    std::vector<int32_t> t(20);
    for (int i = 0; i < 20; i++) t[i] = pose_bin * 20 + i;
    Forest<MPSample> f(engine_, t);
    f.setParam(forest_param(20));
    return f;
  }

  // FaceForest::estimateHeadPose (static, FaceForest.cpp:60-72) with the call's options (step_size,
  // num_head_pose_labels, min_foreground_probability), as getHeadPoseVotesMT uses them.
  static void estimateHeadPose(const ImageSample& sample, const Rect& face_bbox, const Forest<HeadPoseSample>& forest,
                               HeadPoseEstimatorOption options, float* headpose, float* variance) {
    const ffd_rect r{face_bbox.x, face_bbox.y, face_bbox.width, face_bbox.height};
    const ffd_headpose_option o{options.num_head_pose_labels, options.step_size, options.min_foreground_probability};
    std::string err;
    if (detail::engine_call(sample.engine(), err, [&] {
          return ffd_sample_estimate_headpose(sample.handle(), &r, &o, headpose, variance);
        }) != FFD_OK)
      throw std::invalid_argument(err);
    (void)forest;
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
    const std::vector<int32_t> ids = forest.treeIds();
    std::string err;
    if (detail::engine_call(sample.engine(), err, [&] {
          return ffd_sample_estimate_facial_features(sample.handle(), &r, ids.data(), (int32_t)ids.size(), &o, pts);
        }) != FFD_OK)
      throw std::invalid_argument(err);
    ffd_cordinates.clear();
    for (int i = 0; i < options.num_parts && i < FFD_NUM_LANDMARKS; i++) ffd_cordinates.emplace_back(pts[2 * i], pts[2 * i + 1]);
  }

  ffd_engine* engine() const { return engine_; }

 private:
  // The reference-style options: the head-pose tree directory, the FFD forest directories (the given
  // mp_forest_paths plus the sorted sub-directories of mp_forest_param.tree_path, FaceForest.cpp:39-45) and the
  // cascade, converted once into a cached FFDMODEL file keyed by their paths, sizes and modification times.
  bool convert(std::string& model) {
    FaceForestOptions& o = options_;
    for (const std::string& d : detail::subdirs(o.mp_forest_param.tree_path)) o.mp_forest_paths.push_back(d);
    std::sort(o.mp_forest_paths.begin(), o.mp_forest_paths.end());
    std::string key = "hp:" + o.hp_forest_param.tree_path + ":" + std::to_string(o.hp_forest_param.ntrees);
    for (int i = 0; i < o.hp_forest_param.ntrees; i++) {
      char b[32];
      std::snprintf(b, sizeof b, "/tree_%03d.txt", i);
      key += ";" + detail::file_key(o.hp_forest_param.tree_path + b);
    }
    key += "|mp:" + std::to_string(o.mp_forest_param.ntrees);
    for (const std::string& d : o.mp_forest_paths)
      for (int i = 0; i < o.mp_forest_param.ntrees; i++) {
        char b[32];
        std::snprintf(b, sizeof b, "/tree_%03d.txt", i);
        key += ";" + detail::file_key(d + b);
      }
    key += "|fd:" + detail::file_key(o.fd_option.path_face_cascade);
    model = detail::model_cache_path(key);
    if (detail::model_file_ok(model)) return true;
    if (o.fd_option.path_face_cascade.empty()) {  // CascadeClassifier::load("") fails the reference's ctor
      err_ = "(!) Error loading cascade classifier: FaceDetectionOption::path_face_cascade is empty";
      std::fprintf(stderr, "ERROR: %s\n", err_.c_str());
      model.clear();
      return false;
    }
    const ffd_forest_param hp = detail::to_c(o.hp_forest_param), mp = detail::to_c(o.mp_forest_param);
    std::vector<const char*> dirs;
    for (const std::string& d : o.mp_forest_paths) dirs.push_back(d.c_str());
    const char* cascade = o.fd_option.path_face_cascade.c_str();
    if (ffd_model_convert(&hp, &mp, dirs.data(), (int32_t)dirs.size(), cascade, model.c_str()) != FFD_OK) {
      err_ = std::string("(!) Error loading the forests: ") + ffd_model_convert_last_error();
      std::fprintf(stderr, "ERROR: %s\n", err_.c_str());
      model.clear();
      return false;
    }
    return true;
  }
  // the pretrained forests' ForestParam (config_*.txt: face size 125, patch ratio 0.25) unless the options
  // carry the reference's own
  ForestParam forest_param(int ntrees) const {
    ForestParam p = ntrees == 15 ? options_.hp_forest_param : options_.mp_forest_param;
    if (p.face_size <= 0) {
      p.face_size = 125;
      p.patch_size_ratio = 0.25f;
      p.ntrees = ntrees;
      p.features = {0, 1, 2};
    }
    return p;
  }
  static ffd_detect_options detect_options(const FaceDetectionOption& f) {
    ffd_detect_options o;
    ffd_detect_options_init(&o);
    o.min_feature_size = f.min_feature_size;
    o.min_neighbors = f.min_neighbors;
    o.search_scale_factor = f.search_scale_factor;
    return o;
  }
  static void detect(ffd_engine* e, const Mat& img, const FaceDetectionOption& fo, std::vector<Rect>& faces_bboxes) {
    if (!e) throw std::runtime_error("FaceForest not initialised");
    ffd_image im{mat_data(img), img.cols, img.rows, mat_step(img)};
    const ffd_detect_options o = detect_options(fo);
    std::vector<ffd_rect> r(64);
    int32_t n = 0;
    for (int pass = 0; pass < 2; pass++) {
      std::string err;
      if (detail::engine_call(e, err, [&] { return ffd_detect_faces(e, &im, 1, &o, r.data(), nullptr, (int32_t)r.size(), &n); }) != FFD_OK)
        throw std::runtime_error(err);
      if (n <= (int32_t)r.size()) break;
      r.resize(n);
    }
    faces_bboxes.clear();
    for (int32_t i = 0; i < n; i++) faces_bboxes.emplace_back(r[i].x, r[i].y, r[i].width, r[i].height);
  }
  FaceForestOptions options_;
  ffd_engine* engine_ = nullptr;
  std::string err_;
  FaceDetectionOption fd_option_;
  std::vector<ffd_face> out_;  // analyzeFaces' result records (reused across calls)
};

}  // namespace ffd

// Drop-in: the reference's global names, as its headers declare them (FaceForest.hpp, Constants.hpp,
// face_utils.hpp, MeanShift.hpp, Forest.hpp, Tree.hpp, ImageSample.hpp, MPSample.hpp, HeadPoseSample.hpp: the
// forwarding headers of this directory include this one).  FFD_NO_GLOBAL_NAMES keeps everything in namespace ffd.
#ifndef FFD_NO_GLOBAL_NAMES
#ifndef FFD_HAVE_OPENCV
namespace cv {  // the reference spells the image types cv::Mat / cv::Rect / cv::Point (the PODs above without OpenCV)
using ffd::CascadeClassifier;
using ffd::Mat;
using ffd::norm;
using ffd::Point;
using ffd::Point2f;
using ffd::Rect;
}  // namespace cv
#endif
using ffd::CascadeClassifier;
using ffd::Face;
using ffd::FaceAnnotation;
using ffd::FaceDetectionOption;
using ffd::FaceForest;
using ffd::FaceForestOptions;
using ffd::Forest;
using ffd::ForestParam;
using ffd::HeadPoseEstimatorOption;
using ffd::HeadPoseLeaf;
using ffd::HeadPoseSample;
using ffd::ImageSample;
using ffd::MeanShift;
using ffd::MeanShiftOption;
using ffd::MPLeaf;
using ffd::MPSample;
using ffd::MultiPartEstimatorOption;
using ffd::Tree;
using ffd::Vote;
using ffd::areaUnderCurve;
using ffd::enlargeFace;
using ffd::getFacialFeaturesVotesMT;
using ffd::getHeadPoseVotesMT;
using ffd::intersect;
using ffd::loadAnnotations;
using ffd::loadConfigFile;
using ffd::loadImage;
using ffd::NORM_HEADPOSE_VARIANCE_FACTOR;
using ffd::NUM_HEADPOSE_CLASSES;
using ffd::PATCH_CLOSE_TO_FEATURE;
using ffd::TRAIN_IMAGES_PERCENTAGE;
#endif
