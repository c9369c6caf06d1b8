// ffd_convert.cpp — offline converter: reference Boost text archives -> FFDMODEL.
//
// Replaces the run-time archive load of the reference:
//   FaceForest::FaceForest            /root/reference/src/FaceForest.cpp:15-58
//   Forest<S>::load / load_tree       /root/reference/include/Forest.hpp:103-153
//   Tree<S>::load / serialize         /root/reference/include/Tree.hpp:193-237,336-343
//   TreeNode<S>::serialize            /root/reference/include/TreeNode.hpp:150-164
//   ThresholdSplit / SimplePatchFeature serializers
//                                     ThresholdSplit.hpp:60-67, ImageSample.hpp:83-90
//   MPLeaf / HeadPoseLeaf serializers MPSample.hpp:149-158, HeadPoseSample.hpp:154-161
//   loadConfigFile                    /root/reference/src/face_utils.cpp:50-140
// Archive grammar: SURVEY.md Appendix A.  Trees whose i_node != m_num_nodes are
// rejected exactly like Forest::load_tree (Forest.hpp:142-152).
//
// usage: ffd_convert <reference_root> <out.bin>   (built with -DFFD_CONVERT_MAIN)
//   reads <root>/data/config_headpose.txt and <root>/data/config_ffd.txt, then
//   the tree directories they name (relative to <root>); the FFD directory is
//   scanned for sub-directories which are sorted (FaceForest.cpp:39-45).
// The same conversion is in libffd.so as ffd_model_convert (the C++ FaceForest shim runs it for
// reference-style FaceForestOptions: tree directories instead of a converted model).
#include <dirent.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "model_io.hpp"
#include "../../include/ffd.h"

namespace {

struct ForestParam {  // Constants.hpp:24-60
  int max_depth = 15, min_patches = 20, ntests = 250, ntrees = 10, nimages = 500, npatches = 200,
      face_size = 100;
  float patch_size_ratio = 0.25f;
  std::string tree_path, image_path;
  std::vector<int> features;
};

// loadConfigFile (face_utils.cpp:50-140): fixed order of (comment line, value line) pairs.
[[maybe_unused]] bool load_config(const std::string& path, ForestParam& p) {
  std::ifstream f(path);
  if (!f.is_open()) return false;
  std::string line;
  auto next_value = [&](std::string& out) {
    if (!std::getline(f, line)) return false;  // "____..." label line
    if (!std::getline(f, out)) return false;
    while (!out.empty() && (out.back() == '\r' || out.back() == ' ')) out.pop_back();
    return true;
  };
  std::string v;
  if (!next_value(p.image_path)) return false;
  if (!next_value(p.tree_path)) return false;
  if (!next_value(v)) return false;
  p.ntrees = std::stoi(v);
  if (!next_value(v)) return false;
  p.ntests = std::stoi(v);
  if (!next_value(v)) return false;
  p.max_depth = std::stoi(v);
  if (!next_value(v)) return false;
  p.min_patches = std::stoi(v);
  if (!next_value(v)) return false;
  p.nimages = std::stoi(v);
  if (!next_value(v)) return false;
  p.npatches = std::stoi(v);
  if (!next_value(v)) return false;
  p.face_size = std::stoi(v);
  if (!next_value(v)) return false;
  p.patch_size_ratio = std::stof(v);
  if (!next_value(v)) return false;
  std::istringstream ss(v);
  std::string tok;
  while (ss >> tok) p.features.push_back((int)std::stof(tok));  // lexical_cast<float> then int
  return true;
}

// Whitespace tokenizer over a memory-mapped archive.
class Tokens {
 public:
  explicit Tokens(const std::string& path) : path_(path) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("File not found: " + path);
    struct stat st;
    fstat(fd_, &st);
    size_ = (size_t)st.st_size;
    data_ = (const char*)mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (data_ == MAP_FAILED) throw std::runtime_error("mmap failed: " + path);
  }
  ~Tokens() {
    munmap((void*)data_, size_);
    ::close(fd_);
  }
  std::string next() {
    while (pos_ < size_ && isspace((unsigned char)data_[pos_])) pos_++;
    if (pos_ >= size_) throw std::runtime_error("unexpected end of archive " + path_);
    size_t s = pos_;
    while (pos_ < size_ && !isspace((unsigned char)data_[pos_])) pos_++;
    return std::string(data_ + s, pos_ - s);
  }
  long i() {
    std::string t = next();
    char* e = nullptr;
    long v = std::strtol(t.c_str(), &e, 10);
    if (*e) throw std::runtime_error("expected int, got '" + t + "' in " + path_);
    return v;
  }
  float f() {  // text_iarchive reads float via istream >> float (correctly rounded)
    std::string t = next();
    char* e = nullptr;
    float v = std::strtof(t.c_str(), &e);
    if (*e) throw std::runtime_error("expected float, got '" + t + "' in " + path_);
    return v;
  }
  double d() {
    std::string t = next();
    char* e = nullptr;
    double v = std::strtod(t.c_str(), &e);
    if (*e) throw std::runtime_error("expected double, got '" + t + "' in " + path_);
    return v;
  }
  std::string str() {  // length-prefixed string; our paths contain no spaces
    long n = i();
    if (n == 0) return std::string();
    std::string s = next();
    if ((long)s.size() != n) throw std::runtime_error("string length mismatch in " + path_);
    return s;
  }
  void expect(long v, const char* what) {
    long g = i();
    if (g != v)
      throw std::runtime_error(std::string("archive grammar: expected ") + what + " in " + path_);
  }
  bool at_end() {
    while (pos_ < size_ && isspace((unsigned char)data_[pos_])) pos_++;
    return pos_ >= size_;
  }

 private:
  std::string path_;
  int fd_ = -1;
  const char* data_ = nullptr;
  size_t size_ = 0, pos_ = 0;
};

enum Kind { HP, MP };

struct ForestOut {
  std::vector<int64_t> tree_node_off{0}, tree_leaf_off{0};
  std::vector<int32_t> node_leaf;
  std::vector<int16_t> node_split;
  std::vector<int32_t> leaf_n;
  std::vector<float> leaf_fg;
  std::vector<int32_t> hp_labels;
  std::vector<int16_t> mp_offset;
  std::vector<float> mp_var, mp_pf;
  // the fields only the archive writer needs (ffd_archive.cpp, Tree<S>::save Tree.hpp:239-256)
  std::vector<double> node_info;                 // ThresholdSplit::info (0 for leaves)
  std::vector<int64_t> tree_counts;              // per tree: m_num_nodes, i_node
  std::vector<int32_t> tree_param;               // per tree: the archived ForestParam ints (7)
  std::vector<float> tree_ratio;                 // per tree: ForestParam::patch_size_ratio
  std::vector<int32_t> tree_features;            // concatenated ForestParam::features
  std::vector<int64_t> tree_features_off{0};
  std::vector<uint8_t> tree_strings;             // per tree: tree_path, image_path, m_save_path
  std::vector<int64_t> tree_strings_off{0};
};

struct TreeParseState {
  bool first_leaf = true, first_split = true, first_vec_point = true;
  long next_object_id = 0;
  long nodes = 0;
};

void parse_node(Tokens& tk, Kind kind, TreeParseState& st, ForestOut& out, int depth) {
  long oid = tk.i();
  if (oid != st.next_object_id)
    throw std::runtime_error("archive grammar: unexpected object id");
  st.next_object_id++;
  st.nodes++;
  long d = tk.i();
  long is_leaf = tk.i();
  long has_split = tk.i();
  if (d != depth) throw std::runtime_error("archive grammar: depth mismatch");
  int16_t split[FFD_SPLIT_FIELDS] = {0};
  double info = 0.0;
  if (is_leaf) {
    if (st.first_leaf) { tk.expect(0, "leaf class tracking"); tk.expect(0, "leaf class version"); st.first_leaf = false; }
    out.node_leaf.push_back((int32_t)out.leaf_n.size());
    if (kind == HP) {
      out.leaf_n.push_back((int32_t)tk.i());
      out.leaf_fg.push_back(tk.f());
      long cnt = tk.i();
      tk.expect(0, "vector<int> item_version");
      if (cnt != FFD_NUM_HP_LABELS) throw std::runtime_error("HP leaf: expected 5 labels");
      for (long j = 0; j < cnt; j++) out.hp_labels.push_back((int32_t)tk.i());
    } else {
      out.leaf_n.push_back((int32_t)tk.i());
      if (st.first_vec_point) { tk.expect(0, "vector<Point> tracking"); tk.expect(0, "vector<Point> version"); }
      long cnt = tk.i();
      tk.expect(0, "vector<Point> item_version");
      if (st.first_vec_point) { tk.expect(0, "Point tracking"); tk.expect(0, "Point version"); st.first_vec_point = false; }
      if (cnt != FFD_NUM_PARTS) throw std::runtime_error("MP leaf: expected 10 parts");
      for (long j = 0; j < cnt; j++) {
        long x = tk.i(), y = tk.i();
        if (x < -32768 || x > 32767 || y < -32768 || y > 32767) throw std::runtime_error("offset out of int16");
        out.mp_offset.push_back((int16_t)x);
        out.mp_offset.push_back((int16_t)y);
      }
      cnt = tk.i();
      tk.expect(0, "vector<float> item_version");
      if (cnt != FFD_NUM_PARTS) throw std::runtime_error("MP leaf: expected 10 variances");
      for (long j = 0; j < cnt; j++) out.mp_var.push_back(tk.f());
      cnt = tk.i();
      tk.expect(0, "vector<float> item_version");
      if (cnt != FFD_NUM_PARTS) throw std::runtime_error("MP leaf: expected 10 probabilities");
      for (long j = 0; j < cnt; j++) out.mp_pf.push_back(tk.f());
      out.leaf_fg.push_back(tk.f());
    }
  } else {
    out.node_leaf.push_back(-1);
  }
  if (has_split) {
    if (st.first_split) {
      tk.expect(0, "ThresholdSplit tracking"); tk.expect(0, "ThresholdSplit version");
      tk.expect(0, "SimplePatchFeature tracking"); tk.expect(0, "SimplePatchFeature version");
    }
    split[0] = (int16_t)tk.i();  // feature_channel
    if (st.first_split) { tk.expect(0, "Rect tracking"); tk.expect(0, "Rect version"); st.first_split = false; }
    for (int j = 0; j < 8; j++) split[1 + j] = (int16_t)tk.i();  // rect1, rect2 (x y w h)
    info = tk.d();                                                // info (unused at test time; kept for the writer)
    long thr = tk.i();
    if (thr < -32768 || thr > 32767) throw std::runtime_error("threshold out of int16");
    split[9] = (int16_t)thr;
  }
  if (is_leaf && has_split) throw std::runtime_error("node is both leaf and split");
  if (!is_leaf && !has_split) throw std::runtime_error("internal node without split");
  for (int j = 0; j < FFD_SPLIT_FIELDS; j++) out.node_split.push_back(is_leaf ? 0 : split[j]);
  out.node_info.push_back(info);
  if (!is_leaf) {
    tk.expect(3, "TreeNode pointer class id");
    parse_node(tk, kind, st, out, depth + 1);
    tk.expect(3, "TreeNode pointer class id");
    parse_node(tk, kind, st, out, depth + 1);
  }
}

void parse_tree(const std::string& path, Kind kind, ForestOut& out) {
  Tokens tk(path);
  tk.expect(22, "signature length");
  if (tk.next() != "serialization::archive") throw std::runtime_error("not a boost archive: " + path);
  tk.expect(10, "library version");
  tk.expect(0, "Tree tracking");
  tk.expect(0, "Tree version");
  long num_nodes = tk.i(), i_node = tk.i();
  // ForestParam (Constants.hpp:44-59)
  tk.expect(0, "ForestParam tracking");
  tk.expect(0, "ForestParam version");
  for (int j = 0; j < 7; j++) out.tree_param.push_back((int32_t)tk.i());
  out.tree_ratio.push_back(tk.f());
  auto put_str = [&](const std::string& v) {
    out.tree_strings.insert(out.tree_strings.end(), v.begin(), v.end());
    out.tree_strings_off.push_back((int64_t)out.tree_strings.size());
  };
  put_str(tk.str());  // tree_path
  put_str(tk.str());  // image_path
  long nf = tk.i();
  tk.expect(0, "features item_version");
  for (long j = 0; j < nf; j++) out.tree_features.push_back((int32_t)tk.i());
  out.tree_features_off.push_back((int64_t)out.tree_features.size());
  put_str(tk.str());  // m_save_path
  out.tree_counts.push_back(num_nodes);
  out.tree_counts.push_back(i_node);
  // root pointer: class id 3, tracking 1, version 0
  tk.expect(3, "root class id");
  tk.expect(1, "TreeNode tracking");
  tk.expect(0, "TreeNode version");
  TreeParseState st;
  parse_node(tk, kind, st, out, 0);
  if (!tk.at_end()) throw std::runtime_error("trailing tokens in " + path);
  // Tree::isFinished (Tree.hpp:72-79) gate of Forest::load_tree (Forest.hpp:142-152)
  if (i_node != num_nodes) throw std::runtime_error("Tree is not finished successfully: " + path);
  out.tree_node_off.push_back((int64_t)out.node_leaf.size());
  out.tree_leaf_off.push_back((int64_t)out.leaf_n.size());
}

std::vector<std::string> sorted_subdirs(const std::string& dir) {
  std::vector<std::string> v;
  DIR* d = opendir(dir.c_str());
  if (!d) throw std::runtime_error("cannot open directory " + dir);
  while (struct dirent* e = readdir(d)) {
    std::string n = e->d_name;
    if (n == "." || n == "..") continue;
    std::string full = dir + "/" + n;
    struct stat st;
    if (stat(full.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) v.push_back(full);
  }
  closedir(d);
  std::sort(v.begin(), v.end());
  return v;
}

void put_params(ffd::ModelFile& m, const std::string& p, const ForestParam& fp, int n_forests) {
  m.put<int32_t>(p + ".param", "i32", {8},
                 {fp.max_depth, fp.min_patches, fp.ntests, fp.ntrees, fp.nimages, fp.npatches,
                  fp.face_size, n_forests});
  m.put<float>(p + ".patch_ratio", "f32", {1}, {fp.patch_size_ratio});
  std::vector<int32_t> feats(fp.features.begin(), fp.features.end());
  m.put<int32_t>(p + ".features", "i32", {(uint64_t)feats.size()}, feats);
}

void put_forest(ffd::ModelFile& m, const std::string& p, Kind kind, const ForestOut& o) {
  uint64_t T = o.tree_node_off.size() - 1, N = o.node_leaf.size(), L = o.leaf_n.size();
  m.put<int64_t>(p + ".tree_node_off", "i64", {T + 1}, o.tree_node_off);
  m.put<int64_t>(p + ".tree_leaf_off", "i64", {T + 1}, o.tree_leaf_off);
  m.put<int32_t>(p + ".node_leaf", "i32", {N}, o.node_leaf);
  m.put<int16_t>(p + ".node_split", "i16", {N, FFD_SPLIT_FIELDS}, o.node_split);
  m.put<int32_t>(p + ".leaf_n", "i32", {L}, o.leaf_n);
  m.put<float>(p + ".leaf_fg", "f32", {L}, o.leaf_fg);
  if (kind == HP) {
    m.put<int32_t>(p + ".leaf_labels", "i32", {L, FFD_NUM_HP_LABELS}, o.hp_labels);
  } else {
    m.put<int16_t>(p + ".leaf_offset", "i16", {L, FFD_NUM_PARTS, 2}, o.mp_offset);
    m.put<float>(p + ".leaf_var", "f32", {L, FFD_NUM_PARTS}, o.mp_var);
    m.put<float>(p + ".leaf_pf", "f32", {L, FFD_NUM_PARTS}, o.mp_pf);
  }
  m.put<double>(p + ".node_info", "f64", {N}, o.node_info);
  m.put<int64_t>(p + ".tree_counts", "i64", {T, 2}, o.tree_counts);
  m.put<int32_t>(p + ".tree_param", "i32", {T, 7}, o.tree_param);
  m.put<float>(p + ".tree_ratio", "f32", {T}, o.tree_ratio);
  m.put<int32_t>(p + ".tree_features", "i32", {(uint64_t)o.tree_features.size()}, o.tree_features);
  m.put<int64_t>(p + ".tree_features_off", "i64", {T + 1}, o.tree_features_off);
  m.put<uint8_t>(p + ".tree_strings", "u8", {(uint64_t)o.tree_strings.size()}, o.tree_strings);
  m.put<int64_t>(p + ".tree_strings_off", "i64", {3 * T + 1}, o.tree_strings_off);
}

// ---- Haar cascade --------------------------------------------------------
// data/haarcascade_frontalface_alt.xml is in OpenCV's "opencv-cascade-classifier" format (stageType
// BOOST, featureType HAAR), which OpenCV 2.4.9's CascadeClassifier::load reads with
// CascadeClassifier::Data::read + HaarEvaluator::read (objdetect/cascadedetect.cpp); numbers are
// parsed as double (FileNode) and stored as float.  Only stump cascades (one internal node per weak
// classifier, the detector FaceForest.cpp:146 loads) without tilted features are accepted.
struct Cascade {
  int win_w = 0, win_h = 0;
  std::vector<int32_t> stage_first, stage_ntrees, weak_feature, feature_rect;
  std::vector<float> stage_threshold, weak_threshold, weak_leaves, feature_weight;
};

std::string tag_text(const std::string& s, size_t& pos, const std::string& tag, size_t limit) {
  const std::string open = "<" + tag + ">", close = "</" + tag + ">";
  size_t a = s.find(open, pos);
  if (a == std::string::npos || a >= limit) throw std::runtime_error("cascade: missing <" + tag + ">");
  a += open.size();
  size_t b = s.find(close, a);
  if (b == std::string::npos) throw std::runtime_error("cascade: unterminated <" + tag + ">");
  pos = b + close.size();
  return s.substr(a, b - a);
}

std::vector<double> numbers(const std::string& t) {
  std::vector<double> v;
  const char* p = t.c_str();
  char* e = nullptr;
  for (;;) {
    while (*p && isspace((unsigned char)*p)) p++;
    if (!*p) break;
    double d = std::strtod(p, &e);
    if (e == p) throw std::runtime_error("cascade: bad number in '" + t + "'");
    v.push_back(d);
    p = e;
  }
  return v;
}

bool parse_cascade(const std::string& path, Cascade& c) {
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string s = ss.str();
  size_t pos = 0;
  if (tag_text(s, pos, "stageType", s.size()).find("BOOST") == std::string::npos ||
      tag_text(s, pos, "featureType", s.size()).find("HAAR") == std::string::npos)
    throw std::runtime_error("cascade: only BOOST / HAAR cascades are supported");
  c.win_h = (int)numbers(tag_text(s, pos, "height", s.size())).at(0);
  c.win_w = (int)numbers(tag_text(s, pos, "width", s.size())).at(0);
  size_t st = s.find("<stages>", pos), st_end = s.find("</stages>", pos);
  size_t ft = s.find("<features>", pos), ft_end = s.find("</features>", pos);
  if (st == std::string::npos || st_end == std::string::npos || ft == std::string::npos || ft_end == std::string::npos)
    throw std::runtime_error("cascade: missing <stages> or <features>");
  // stages: <maxWeakCount> <stageThreshold> <weakClassifiers> (<internalNodes> <leafValues>)*
  pos = st;
  for (;;) {
    size_t nxt = s.find("<maxWeakCount>", pos);
    if (nxt == std::string::npos || nxt > st_end) break;
    pos = nxt;
    (void)tag_text(s, pos, "maxWeakCount", st_end);
    c.stage_threshold.push_back((float)numbers(tag_text(s, pos, "stageThreshold", st_end)).at(0));
    size_t wc_end = s.find("</weakClassifiers>", pos);
    if (wc_end == std::string::npos || wc_end > st_end) throw std::runtime_error("cascade: bad <weakClassifiers>");
    c.stage_first.push_back((int32_t)c.weak_feature.size());
    int n = 0;
    for (;;) {
      size_t in = s.find("<internalNodes>", pos);
      if (in == std::string::npos || in > wc_end) break;
      pos = in;
      std::vector<double> nd = numbers(tag_text(s, pos, "internalNodes", wc_end));
      std::vector<double> lv = numbers(tag_text(s, pos, "leafValues", wc_end));
      if (nd.size() != 4 || lv.size() != 2)
        throw std::runtime_error("cascade: only stump classifiers (one internal node, two leaves) are supported");
      c.weak_feature.push_back((int32_t)nd[2]);
      c.weak_threshold.push_back((float)nd[3]);
      c.weak_leaves.push_back((float)lv[0]);
      c.weak_leaves.push_back((float)lv[1]);
      n++;
    }
    c.stage_ntrees.push_back(n);
    pos = wc_end;
  }
  // features: <_> <rects> (<_> x y w h weight </_>){2,3} </rects> [<tilted>t</tilted>] </_>
  pos = ft;
  for (;;) {
    size_t r = s.find("<rects>", pos);
    if (r == std::string::npos || r > ft_end) break;
    size_t r_end = s.find("</rects>", r);
    int k = 0;
    int32_t rect[12] = {0};
    float w[3] = {0.f, 0.f, 0.f};
    pos = r + 7;
    for (;;) {
      size_t a = s.find("<_>", pos);
      if (a == std::string::npos || a > r_end) break;
      size_t b = s.find("</_>", a);
      std::vector<double> v = numbers(s.substr(a + 3, b - a - 3));
      if (v.size() != 5 || k >= 3) throw std::runtime_error("cascade: bad feature rectangle");
      for (int j = 0; j < 4; j++) rect[4 * k + j] = (int32_t)v[j];
      w[k] = (float)v[4];
      k++;
      pos = b + 4;
    }
    if (k < 2) throw std::runtime_error("cascade: feature with fewer than 2 rectangles");
    pos = r_end + 8;
    size_t tl = s.find("<tilted>", pos), next_r = s.find("<rects>", pos);
    if (tl != std::string::npos && tl < ft_end && (next_r == std::string::npos || tl < next_r) &&
        numbers(tag_text(s, tl, "tilted", ft_end)).at(0) != 0)
      throw std::runtime_error("cascade: tilted features are not supported");
    c.feature_rect.insert(c.feature_rect.end(), rect, rect + 12);
    c.feature_weight.insert(c.feature_weight.end(), w, w + 3);
  }
  const int nf = (int)c.feature_weight.size() / 3;
  for (int32_t fi : c.weak_feature)
    if (fi < 0 || fi >= nf) throw std::runtime_error("cascade: feature index out of range");
  return true;
}

void put_cascade(ffd::ModelFile& m, const Cascade& c) {
  const uint64_t S = c.stage_threshold.size(), C = c.weak_feature.size(), F = c.feature_weight.size() / 3;
  m.put<int32_t>("haar.window", "i32", {2}, {c.win_w, c.win_h});
  m.put<int32_t>("haar.stage_first", "i32", {S}, c.stage_first);
  m.put<int32_t>("haar.stage_ntrees", "i32", {S}, c.stage_ntrees);
  m.put<float>("haar.stage_threshold", "f32", {S}, c.stage_threshold);
  m.put<int32_t>("haar.weak_feature", "i32", {C}, c.weak_feature);
  m.put<float>("haar.weak_threshold", "f32", {C}, c.weak_threshold);
  m.put<float>("haar.weak_leaves", "f32", {C, 2}, c.weak_leaves);
  m.put<int32_t>("haar.feature_rect", "i32", {F, 3, 4}, c.feature_rect);
  m.put<float>("haar.feature_weight", "f32", {F, 3}, c.feature_weight);
}


// Convert the archives of one head-pose forest (hp.ntrees trees in hp_dir, Forest::load Forest.hpp:116-127)
// and of the pose-conditional FFD forests (mp.ntrees trees in each of mp_dirs, already in the reference's
// sorted order, FaceForest.cpp:39-55) plus an optional Haar cascade into an FFDMODEL file.
std::string convert_model(const ForestParam& hp, const std::string& hp_dir, const ForestParam& mp,
                          const std::vector<std::string>& mp_dirs, const std::string& cascade_xml,
                          const std::string& outp) {
  ffd::ModelFile m;
  ForestOut hpo;
  char buf[4096];
  for (int i = 0; i < hp.ntrees; i++) {  // Forest::load (Forest.hpp:116-127)
    std::snprintf(buf, sizeof buf, "%s/tree_%03d.txt", hp_dir.c_str(), i);
    parse_tree(buf, HP, hpo);
  }
  put_params(m, "hp", hp, 1);
  put_forest(m, "hp", HP, hpo);
  if (mp_dirs.empty()) throw std::runtime_error("no FFD forest directories");
  ForestOut mpo;
  for (auto& d : mp_dirs)
    for (int i = 0; i < mp.ntrees; i++) {
      std::snprintf(buf, sizeof buf, "%s/tree_%03d.txt", d.c_str(), i);
      parse_tree(buf, MP, mpo);
    }
  put_params(m, "mp", mp, (int)mp_dirs.size());
  put_forest(m, "mp", MP, mpo);
  Cascade cas;  // FaceDetectionOption::path_face_cascade as demo.cpp:186 / eval_ffd.cpp:143 set it
  // a cascade that is named but cannot be read fails the conversion, as CascadeClassifier::load fails the
  // reference's constructor (FaceForest.cpp:23-27)
  const bool have_cascade = !cascade_xml.empty();
  if (have_cascade && !parse_cascade(cascade_xml, cas)) throw std::runtime_error("cannot open the cascade " + cascade_xml);
  if (have_cascade) put_cascade(m, cas);
  // a temporary name of this process and call, renamed over the target (atomic on one file system), so
  // concurrent conversions of the same directories (one per rank) never interleave their writes
  static std::atomic<unsigned> seq{0};
  const std::string tmp = outp + ".tmp." + std::to_string((long)getpid()) + "." + std::to_string(seq++);
  try {
    m.save(tmp);
  } catch (...) {
    std::remove(tmp.c_str());
    throw;
  }
  if (std::rename(tmp.c_str(), outp.c_str()) != 0) {
    std::remove(tmp.c_str());
    throw std::runtime_error("rename failed: " + outp);
  }
  std::string msg = "hp " + std::to_string(hpo.tree_node_off.size() - 1) + " trees " +
                    std::to_string(hpo.node_leaf.size()) + " nodes " + std::to_string(hpo.leaf_n.size()) +
                    " leaves; mp " + std::to_string(mp_dirs.size()) + " forests " +
                    std::to_string(mpo.tree_node_off.size() - 1) + " trees " + std::to_string(mpo.node_leaf.size()) +
                    " nodes " + std::to_string(mpo.leaf_n.size()) + " leaves -> " + outp;
  if (have_cascade)
    msg += "\nhaar cascade " + std::to_string(cas.win_w) + "x" + std::to_string(cas.win_h) + ", " +
           std::to_string(cas.stage_threshold.size()) + " stages, " + std::to_string(cas.weak_feature.size()) +
           " weak classifiers, " + std::to_string(cas.feature_weight.size() / 3) + " features";
  return msg;
}

thread_local std::string g_convert_error;

}  // namespace

namespace ffd_host {
void cascade_arrays(const std::string& xml, ffd::ModelFile& m);  // (declared in ffd_engine_impl.hpp)
}
// ffd_detector_create's cascade: the XML as the "haar.*" arrays ffd_convert writes
void ffd_host::cascade_arrays(const std::string& xml, ffd::ModelFile& m) {
  Cascade c;
  if (!parse_cascade(xml, c)) throw std::runtime_error("cannot open the cascade " + xml);
  put_cascade(m, c);
}

namespace {

ForestParam from_c(const ffd_forest_param& c) {
  ForestParam p;
  p.max_depth = c.max_depth; p.min_patches = c.min_patches; p.ntests = c.ntests; p.ntrees = c.ntrees;
  p.nimages = c.nimages; p.npatches = c.npatches; p.face_size = c.face_size;
  p.patch_size_ratio = c.patch_size_ratio;
  p.tree_path = c.tree_path ? c.tree_path : "";
  p.image_path = c.image_path ? c.image_path : "";
  for (int i = 0; i < c.n_features; i++) p.features.push_back(c.features[i]);
  return p;
}

}  // namespace

extern "C" {

ffd_status ffd_model_convert(const ffd_forest_param* hp, const ffd_forest_param* mp, const char* const* mp_dirs,
                             int32_t n_mp_dirs, const char* cascade_xml, const char* out_path) {
  if (!hp || !mp || !out_path || !hp->tree_path || n_mp_dirs < 0 || (n_mp_dirs && !mp_dirs) ||
      (hp->n_features && !hp->features) || (mp->n_features && !mp->features)) {
    g_convert_error = "bad arguments";
    return FFD_ERR_INVALID_ARGUMENT;
  }
  try {
    std::vector<std::string> dirs;
    for (int i = 0; i < n_mp_dirs; i++) dirs.push_back(mp_dirs[i]);
    (void)convert_model(from_c(*hp), hp->tree_path, from_c(*mp), dirs, cascade_xml ? cascade_xml : "", out_path);
    return FFD_OK;
  } catch (const std::exception& e) {
    g_convert_error = e.what();
    return FFD_ERR_MODEL;
  }
}

const char* ffd_model_convert_last_error(void) { return g_convert_error.c_str(); }

ffd_status ffd_forest_subdirs(const char* dir, char* buf, int64_t cap, int64_t* size) {
  if (!dir || !size) {
    g_convert_error = "bad arguments";
    return FFD_ERR_INVALID_ARGUMENT;
  }
  try {
    std::string all;
    for (auto& d : sorted_subdirs(dir)) {
      all += d;
      all.push_back('\0');
    }
    *size = (int64_t)all.size();
    if (buf) {
      if (cap < (int64_t)all.size()) {
        g_convert_error = "buffer too small";
        return FFD_ERR_INVALID_ARGUMENT;
      }
      std::memcpy(buf, all.data(), all.size());
    }
    return FFD_OK;
  } catch (const std::exception& e) {
    g_convert_error = e.what();
    return FFD_ERR_MODEL;
  }
}

}  // extern "C"

#ifdef FFD_CONVERT_MAIN
// usage: ffd_convert <reference_root> <out.bin>: the configs and tree directories the reference's mains use
// (eval_ffd.cpp:137-143), relative to <reference_root>.
int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: %s <reference_root> <out.bin>\n", argv[0]);
    return 2;
  }
  std::string root = argv[1], outp = argv[2];
  try {
    ForestParam hp, mp;
    if (!load_config(root + "/data/config_headpose.txt", hp))
      throw std::runtime_error("cannot parse config_headpose.txt");
    if (!load_config(root + "/data/config_ffd.txt", mp))
      throw std::runtime_error("cannot parse config_ffd.txt");
    std::string cascade = root + "/data/haarcascade_frontalface_alt.xml";  // (a tree without one: no detector)
    struct stat cst;
    if (stat(cascade.c_str(), &cst) != 0) cascade.clear();
    const std::string msg = convert_model(hp, root + "/" + hp.tree_path, mp, sorted_subdirs(root + "/" + mp.tree_path),
                                          cascade, outp);
    std::printf("ffd_convert: %s\n", msg.c_str());
  } catch (const std::exception& e) {
    std::fprintf(stderr, "ffd_convert: ERROR: %s\n", e.what());
    return 1;
  }
  return 0;
}
#endif
