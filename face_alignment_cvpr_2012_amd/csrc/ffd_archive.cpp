// ffd_archive.cpp — Boost text-archive writer for the converted forests.
//
// Re-emits one tree of an FFDMODEL container (include/ffd_model_format.h) as the bytes the
// reference's Tree<S>::save writes (/root/reference/include/Tree.hpp:239-256: text_oarchive of
// *this), so trees held or produced here can be loaded by the reference's Forest<S>::load
// (Forest.hpp:103-153).  The token grammar is SURVEY.md Appendix A; the serializers it follows:
//   Tree<S>::serialize          Tree.hpp:336-343      m_num_nodes, i_node, m_param, m_save_path, root
//   ForestParam::serialize      Constants.hpp:44-59   7 ints, ratio, tree_path, image_path, features
//   TreeNode<S>::serialize      TreeNode.hpp:150-164  depth, is_leaf, has_split, [leaf], [split], left, right
//   ThresholdSplit::serialize   ThresholdSplit.hpp:60-67  feature, info, threshold
//   SimplePatchFeature          ImageSample.hpp:83-90     channel, rect1, rect2
//   cv::Rect / cv::Point        opencv_serialization.hpp:65-79
//   MPLeaf::serialize           MPSample.hpp:149-158
//   HeadPoseLeaf::serialize     HeadPoseSample.hpp:154-161
// Boost text_oarchive conventions reproduced here (library version 10):
//   * tokens are separated by one space; a newline precedes every tracked object (each TreeNode's
//     object id); the archive does not end with a newline;
//   * class information ("tracking version", here always "0 0") is written at the first occurrence
//     of a class in the archive only; a pointer to TreeNode writes its class id "3", followed at
//     the first occurrence (the root) by "1 0" (tracked, version 0);
//   * float with precision digits10 + 2 = 8, double with 17 (default float field, i.e. %.8g /
//     %.17g); std::vector writes count, item_version (0), items; std::string writes length, text.
// The archive-only fields (split info, the archived ForestParam and paths, node counters) come from
// the converter; a container without them (a synthetic forest, ffd_synth_forest) gets the values a
// freshly grown tree would carry: info 0, i_node = m_num_nodes = its node count, the container's
// ForestParam, and paths "tree_%03d.txt".
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "ffd.h"
#include "model_io.hpp"

struct ffd_model {
  ffd::ModelFile file;
};

namespace {

thread_local std::string g_model_error;

ffd_status fail(ffd_status s, const std::string& msg) {
  g_model_error = msg;
  return s;
}

const char* prefix_of(int32_t kind) { return kind == FFD_FOREST_HEADPOSE ? "hp" : kind == FFD_FOREST_FFD ? "mp" : nullptr; }

class Writer {
 public:
  explicit Writer(std::string& out) : out_(out) {}
  void tok(const char* s) {
    if (!first_) out_.push_back(pending_nl_ ? '\n' : ' ');
    first_ = false;
    pending_nl_ = false;
    out_.append(s);
  }
  void i(long long v) {
    char b[32];
    std::snprintf(b, sizeof b, "%lld", v);
    tok(b);
  }
  void f(float v) {  // text_oprimitive: precision std::numeric_limits<float>::digits10 + 2
    char b[48];
    std::snprintf(b, sizeof b, "%.8g", (double)v);
    tok(b);
  }
  void d(double v) {  // precision std::numeric_limits<double>::digits10 + 2
    char b[48];
    std::snprintf(b, sizeof b, "%.17g", v);
    tok(b);
  }
  void str(const uint8_t* s, size_t n) {
    i((long long)n);
    tok(std::string(reinterpret_cast<const char*>(s), n).c_str());
  }
  void newline() { pending_nl_ = true; }

 private:
  std::string& out_;
  bool first_ = true, pending_nl_ = false;
};

struct TreeView {
  int kind = 0;
  const int32_t* node_leaf = nullptr;
  const int16_t* node_split = nullptr;
  const double* node_info = nullptr;
  const int32_t* leaf_n = nullptr;
  const float* leaf_fg = nullptr;
  const int32_t* hp_labels = nullptr;
  const int16_t* mp_offset = nullptr;
  const float* mp_var = nullptr;
  const float* mp_pf = nullptr;
  int64_t n0 = 0, n1 = 0;  // node range [n0, n1)
};

struct EmitState {
  bool first_leaf = true, first_split = true, first_point = true;
  long long next_oid = 0;
};

// One TreeNode in pre-order (TreeNode.hpp:150-164); returns the next node index.
int64_t emit_node(Writer& w, const TreeView& t, int64_t n, int depth, EmitState& st) {
  if (n >= t.n1) throw std::runtime_error("tree structure runs past its node range");
  const bool leaf = t.node_leaf[n] >= 0;
  w.newline();
  w.i(st.next_oid++);
  w.i(depth);
  w.i(leaf ? 1 : 0);
  w.i(leaf ? 0 : 1);  // has_split (the converter admits exactly one of the two)
  if (leaf) {
    const int64_t l = t.node_leaf[n];
    if (st.first_leaf) { w.i(0); w.i(0); st.first_leaf = false; }
    if (t.kind == FFD_FOREST_HEADPOSE) {  // HeadPoseSample.hpp:154-161
      w.i(t.leaf_n[l]);
      w.f(t.leaf_fg[l]);
      w.i(FFD_NUM_HP_LABELS);
      w.i(0);
      for (int j = 0; j < FFD_NUM_HP_LABELS; j++) w.i(t.hp_labels[l * FFD_NUM_HP_LABELS + j]);
    } else {  // MPSample.hpp:149-158
      w.i(t.leaf_n[l]);
      if (st.first_point) { w.i(0); w.i(0); }  // vector<cv::Point> class info
      w.i(FFD_NUM_PARTS);
      w.i(0);
      if (st.first_point) { w.i(0); w.i(0); st.first_point = false; }  // cv::Point class info
      for (int j = 0; j < FFD_NUM_PARTS; j++) {
        w.i(t.mp_offset[(l * FFD_NUM_PARTS + j) * 2 + 0]);
        w.i(t.mp_offset[(l * FFD_NUM_PARTS + j) * 2 + 1]);
      }
      w.i(FFD_NUM_PARTS);
      w.i(0);
      for (int j = 0; j < FFD_NUM_PARTS; j++) w.f(t.mp_var[l * FFD_NUM_PARTS + j]);
      w.i(FFD_NUM_PARTS);
      w.i(0);
      for (int j = 0; j < FFD_NUM_PARTS; j++) w.f(t.mp_pf[l * FFD_NUM_PARTS + j]);
      w.f(t.leaf_fg[l]);
    }
    return n + 1;
  }
  const int16_t* s = t.node_split + n * FFD_SPLIT_FIELDS;
  if (st.first_split) { w.i(0); w.i(0); w.i(0); w.i(0); }  // ThresholdSplit, SimplePatchFeature
  w.i(s[0]);                                                   // feature_channel
  if (st.first_split) { w.i(0); w.i(0); st.first_split = false; }  // cv::Rect
  for (int j = 1; j <= 8; j++) w.i(s[j]);
  w.d(t.node_info ? t.node_info[n] : 0.0);
  w.i(s[9]);
  w.i(3);  // left child pointer: class id
  int64_t next = emit_node(w, t, n + 1, depth + 1, st);
  w.i(3);  // right child pointer
  return emit_node(w, t, next, depth + 1, st);
}

template <typename T>
const T* opt(const ffd::ModelFile& m, const std::string& name) {
  return m.has(name) ? m.get(name).as<T>() : nullptr;
}

ffd_status archive_tree(const ffd::ModelFile& m, int32_t kind, int32_t tree, std::string& out) {
  const char* p = prefix_of(kind);
  if (!p) return fail(FFD_ERR_INVALID_ARGUMENT, "forest_kind must be FFD_FOREST_HEADPOSE or FFD_FOREST_FFD");
  const std::string P = p;
  try {
    const auto& toff = m.get(P + ".tree_node_off");
    const int64_t T = (int64_t)toff.count() - 1;
    if (tree < 0 || tree >= T) return fail(FFD_ERR_INVALID_ARGUMENT, "tree index out of range");
    TreeView t;
    t.kind = kind;
    t.node_leaf = m.get(P + ".node_leaf").as<int32_t>();
    t.node_split = m.get(P + ".node_split").as<int16_t>();
    t.node_info = opt<double>(m, P + ".node_info");
    t.leaf_n = m.get(P + ".leaf_n").as<int32_t>();
    t.leaf_fg = m.get(P + ".leaf_fg").as<float>();
    if (kind == FFD_FOREST_HEADPOSE) {
      t.hp_labels = m.get(P + ".leaf_labels").as<int32_t>();
    } else {
      t.mp_offset = m.get(P + ".leaf_offset").as<int16_t>();
      t.mp_var = m.get(P + ".leaf_var").as<float>();
      t.mp_pf = m.get(P + ".leaf_pf").as<float>();
    }
    t.n0 = toff.as<int64_t>()[tree];
    t.n1 = toff.as<int64_t>()[tree + 1];

    const int64_t* counts = opt<int64_t>(m, P + ".tree_counts");
    const int32_t* tparam = opt<int32_t>(m, P + ".tree_param");
    const float* tratio = opt<float>(m, P + ".tree_ratio");
    const int32_t* tfeat = opt<int32_t>(m, P + ".tree_features");
    const int64_t* tfeat_off = opt<int64_t>(m, P + ".tree_features_off");
    const uint8_t* tstr = opt<uint8_t>(m, P + ".tree_strings");
    const int64_t* tstr_off = opt<int64_t>(m, P + ".tree_strings_off");

    out.clear();
    out.reserve((size_t)(t.n1 - t.n0) * 48 + 256);
    Writer w(out);
    // boost::archive::text_oarchive header
    w.i(22);
    w.tok("serialization::archive");
    w.i(10);
    // Tree<S> (class info, first occurrence)
    w.i(0);
    w.i(0);
    w.i(counts ? counts[2 * tree] : t.n1 - t.n0);      // m_num_nodes
    w.i(counts ? counts[2 * tree + 1] : t.n1 - t.n0);  // i_node
    // ForestParam (Constants.hpp:44-59)
    w.i(0);
    w.i(0);
    const int32_t* fp = tparam ? tparam + 7 * tree : m.get(P + ".param").as<int32_t>();
    for (int j = 0; j < 7; j++) w.i(fp[j]);
    w.f(tratio ? tratio[tree] : m.get(P + ".patch_ratio").as<float>()[0]);
    char dflt[64];
    std::snprintf(dflt, sizeof dflt, "tree_%03d.txt", tree);
    auto put_string = [&](int j, const char* fallback) {
      if (tstr && tstr_off) {
        const int64_t a = tstr_off[3 * tree + j], b = tstr_off[3 * tree + j + 1];
        w.str(tstr + a, (size_t)(b - a));
      } else {
        w.str(reinterpret_cast<const uint8_t*>(fallback), std::strlen(fallback));
      }
    };
    put_string(0, "trees");   // tree_path
    put_string(1, "images");  // image_path
    if (tfeat && tfeat_off) {
      const int64_t a = tfeat_off[tree], b = tfeat_off[tree + 1];
      w.i(b - a);
      w.i(0);
      for (int64_t j = a; j < b; j++) w.i(tfeat[j]);
    } else {
      const auto& fa = m.get(P + ".features");
      w.i((long long)fa.count());
      w.i(0);
      for (uint64_t j = 0; j < fa.count(); j++) w.i(fa.as<int32_t>()[j]);
    }
    put_string(2, dflt);  // m_save_path
    // root: TreeNode* (class id 3, first occurrence: tracked, version 0)
    w.i(3);
    w.i(1);
    w.i(0);
    EmitState st;
    const int64_t end = emit_node(w, t, t.n0, 0, st);
    if (end != t.n1) return fail(FFD_ERR_MODEL, "tree's pre-order does not cover its node range");
  } catch (const std::exception& e) {
    return fail(FFD_ERR_MODEL, e.what());
  }
  return FFD_OK;
}

ffd_status archive_tree(const ffd_model* model, int32_t kind, int32_t tree, std::string& out) {
  if (!model) return fail(FFD_ERR_INVALID_ARGUMENT, "model is NULL");
  return archive_tree(model->file, kind, tree, out);
}

}  // namespace

namespace ffd_host {
// Boost text archive of tree `tree` of an in-memory FFDMODEL container (trained trees, ffd_train.cpp)
ffd_status archive_model_tree(const ffd::ModelFile& m, int32_t kind, int32_t tree, std::string& out, std::string& err) {
  const ffd_status st = archive_tree(m, kind, tree, out);
  if (st != FFD_OK) err = g_model_error;
  return st;
}
}  // namespace ffd_host

extern "C" {

ffd_status ffd_model_open(const char* path, ffd_model** out) {
  if (!path || !out) return fail(FFD_ERR_INVALID_ARGUMENT, "path and out must be non-NULL");
  *out = nullptr;
  auto* m = new (std::nothrow) ffd_model;
  if (!m) return fail(FFD_ERR_OUT_OF_MEMORY, "out of host memory");
  try {
    m->file.load(path);
    m->file.get("hp.tree_node_off");
    m->file.get("mp.tree_node_off");
  } catch (const std::exception& e) {
    delete m;
    return fail(FFD_ERR_MODEL, e.what());
  }
  *out = m;
  return FFD_OK;
}

void ffd_model_close(ffd_model* model) { delete model; }

const char* ffd_model_last_error(void) { return g_model_error.c_str(); }

int32_t ffd_model_num_trees(const ffd_model* model, int32_t forest_kind) {
  const char* p = prefix_of(forest_kind);
  if (!model || !p) return -1;
  return (int32_t)model->file.get(std::string(p) + ".tree_node_off").count() - 1;
}

ffd_status ffd_model_tree_save_path(const ffd_model* model, int32_t forest_kind, int32_t tree, char* buf, int32_t cap) {
  const char* p = prefix_of(forest_kind);
  if (!model || !p || !buf || cap <= 0) return fail(FFD_ERR_INVALID_ARGUMENT, "bad argument");
  if (tree < 0 || tree >= ffd_model_num_trees(model, forest_kind)) return fail(FFD_ERR_INVALID_ARGUMENT, "tree index out of range");
  const std::string P = p;
  std::string s;
  if (model->file.has(P + ".tree_strings") && model->file.has(P + ".tree_strings_off")) {
    const int64_t* off = model->file.get(P + ".tree_strings_off").as<int64_t>();
    const uint8_t* str = model->file.get(P + ".tree_strings").as<uint8_t>();
    s.assign(reinterpret_cast<const char*>(str + off[3 * tree + 2]), (size_t)(off[3 * tree + 3] - off[3 * tree + 2]));
  } else {
    char d[64];
    std::snprintf(d, sizeof d, "tree_%03d.txt", tree);
    s = d;
  }
  if ((int32_t)s.size() >= cap) return fail(FFD_ERR_INVALID_ARGUMENT, "buffer too small");
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return FFD_OK;
}

ffd_status ffd_model_tree_archive(const ffd_model* model, int32_t forest_kind, int32_t tree, char* buf, int64_t cap,
                                  int64_t* size) {
  if (!size) return fail(FFD_ERR_INVALID_ARGUMENT, "size must be non-NULL");
  std::string s;
  ffd_status st = archive_tree(model, forest_kind, tree, s);
  if (st != FFD_OK) return st;
  *size = (int64_t)s.size();
  if (!buf) return FFD_OK;  // size query
  if (cap < (int64_t)s.size()) return fail(FFD_ERR_INVALID_ARGUMENT, "buffer too small");
  std::memcpy(buf, s.data(), s.size());
  return FFD_OK;
}

ffd_status ffd_model_save_tree(const ffd_model* model, int32_t forest_kind, int32_t tree, const char* path) {
  if (!path) return fail(FFD_ERR_INVALID_ARGUMENT, "path must be non-NULL");
  std::string s;
  ffd_status st = archive_tree(model, forest_kind, tree, s);
  if (st != FFD_OK) return st;
  FILE* f = std::fopen(path, "wb");
  if (!f) return fail(FFD_ERR_INVALID_ARGUMENT, std::string("cannot write ") + path);
  const bool ok = std::fwrite(s.data(), 1, s.size(), f) == s.size();
  if (std::fclose(f) != 0 || !ok) return fail(FFD_ERR_INTERNAL, std::string("write failed: ") + path);
  return FFD_OK;
}

}  // extern "C"
