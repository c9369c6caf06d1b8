// ffd_engine_impl.hpp — host-side engine state shared by the translation units of libffd.so
// (ffd_engine.cpp: model, pipeline and the single-device C ABI; ffd_group.cpp: multi-device and
// RCCL).  Not installed: the public interface is include/ffd.h.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../include/ffd.h"
#include "ffd_device.hpp"
#include "ffd_haar.hpp"
#include "ffd_kernels.hpp"

namespace ffd {
class ModelFile;  // model_io.hpp
}

namespace ffd_host {

using namespace ffd;

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct DeviceOom : HipError {  // hipMalloc found no room: FFD_ERR_OUT_OF_MEMORY, not FFD_ERR_DEVICE
  using HipError::HipError;
};
struct Unsupported : std::runtime_error {  // an input outside what the engine computes exactly: FFD_ERR_UNSUPPORTED
  using std::runtime_error::runtime_error;
};

#define HIP_CHECK(expr)                                                                        \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      throw HipError(std::string(#expr) + ": " + hipGetErrorString(e_) + " (" __FILE__ ":" +  \
                     std::to_string(__LINE__) + ")");                                         \
  } while (0)

// Device buffer that grows on demand (never shrinks).
struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  ~DevBuf() { if (p) (void)hipFree(p); }
  void* ensure(size_t bytes) {
    if (bytes <= n) return p;
    if (p) { (void)hipFree(p); p = nullptr; n = 0; }
    size_t want = std::max<size_t>(bytes, 256);
    const hipError_t r = hipMalloc(&p, want);
    if (r == hipErrorOutOfMemory) {
      (void)hipGetLastError();  // (clear the sticky error)
      p = nullptr;
      throw DeviceOom("device allocation of " + std::to_string(want) + " bytes failed (out of memory)");
    }
    HIP_CHECK(r);
    n = want;
    return p;
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

template <class T> void upload(DevBuf& b, const std::vector<T>& v, hipStream_t s) {
  b.ensure(v.size() * sizeof(T));
  if (!v.empty()) HIP_CHECK(hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
}

inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

struct Geometry {
  int W = 0, H = 0, nhx = 0, nhy = 0, nmx = 0, nmy = 0;
  float scale = 0;
};

// The leaf offsets a vote table's voting parts can add to a patch centre (per axis, inclusive)
struct VoteRange {
  bool any = false;  // no voting offset at all: no votes
  int lo_x = 0, hi_x = 0, lo_y = 0, hi_y = 0;
};

// 1: some vote position of face f may leave int16 (FaceDesc::wide: 16-B VoteW lists); positions are
// vox + xi step + half + off_x, voy + yi step_y + half + off_y (face_utils.cpp:257-293)
inline int votes_wide(const ffd::FaceDesc& f, int step, int step_y, int half, const VoteRange& r) {
  if (!r.any || f.nmx <= 0 || f.nmy <= 0) return 0;
  const int64_t x0 = (int64_t)f.vox + half + r.lo_x, x1 = (int64_t)f.vox + half + (int64_t)(f.nmx - 1) * step + r.hi_x;
  const int64_t y0 = (int64_t)f.voy + half + r.lo_y, y1 = (int64_t)f.voy + half + (int64_t)(f.nmy - 1) * step_y + r.hi_y;
  return x0 < -32768 || y0 < -32768 || x1 > 32767 || y1 > 32767;
}

}  // namespace ffd_host

using namespace ffd;  // internal header: the engine's TUs work in ffd's vocabulary
using ffd_host::DevBuf;
using ffd_host::Geometry;
using ffd_host::HipError;
using ffd_host::DeviceOom;
using ffd_host::upload;

// Per-stream workspace: a chunk of faces runs its whole pipeline on one stream; consecutive
// chunks alternate streams so one chunk's memory-bound traversal overlaps the next chunk's
// VALU-bound Gabor stage, and a chunk's channel planes stay in the Infinity Cache between the
// kernel that writes them and the traversals that read them.
struct Workspace {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  // channel-stage fork: the five Gabor kernels and k_integral are independent, so they are spread
  // over `stream` and these streams (joined back before the head-pose traversal)
  std::vector<hipStream_t> fork;
  std::vector<hipEvent_t> fork_ev;  // [0]: gray ready; [1 + i]: fork stream i done
  bool pending = false;
  DevBuf faces, gray, mag, chan, hpleaf, mpleaf, votes, state, ms_mean, vote_counts;
  DevBuf gabor_redo;  // per scale and face: the fast Gabor instance flags faces for the exact one
  DevBuf ms_order;    // MeanShift chains sorted by list length (k_ms_order)
  DevBuf gabor_mm;    // per face and scale: the banded Gabor instances' 16-word slots (zero between launches)
  std::vector<FaceDesc> h_fds;  // host staging, reused only after `done`
  std::vector<FaceDesc> desc;   // descriptors of the chunk last run here (ffd_get_trace)
  int first = 0, count = 0;
  ~Workspace() {
    for (auto e : fork_ev) (void)hipEventDestroy(e);
    for (auto f : fork) (void)hipStreamDestroy(f);
    if (done) (void)hipEventDestroy(done);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

namespace ffd_host {
// Re-encode breadth-first 16-byte nodes (children adjacent) as k_traverse's 16-byte pair records
// in depth-first order (ffd_device.hpp "pair records"); roots_out[t] = tree t's root pair.
void build_pair_records(const std::vector<uint4>& bfs, const std::vector<int32_t>& roots, std::vector<uint4>& out,
                        std::vector<int32_t>& roots_out, std::vector<uint32_t>& far);
// Heap-ordered tree tops (ffd_device.hpp "tree tops") of every tree: TOP_CAP records + pair indices.
void build_tree_tops(const std::vector<uint4>& pairs, const std::vector<int32_t>& proots,
                     const std::vector<uint32_t>& far, std::vector<uint4>& tops, std::vector<uint32_t>& top_idx);
}  // namespace ffd_host

struct ffd_engine {
  std::string err;
  int device = 0;
  ffd_engine_desc desc{};
  int max_chunk = 4096;
  DevBuf sample_hs;          // the FFD tree list of the last image-sample grid evaluation (ffd_sample_eval_grid)
  HpState sample_hs_host{};  // ... and its host copy (uploaded again only when a call's list differs)
  int64_t chunk_bytes = (int64_t)40 << 30;  // a chunk's face buffers at most (FFD_CHUNK_BYTES; C2's 4,096 faces: ~26 GB)
  bool detector_only = false;  // ffd_detector_create: a Haar cascade and no forests
  int n_streams = 1;
  int gabor_exact = 0;      // FFD_GABOR_EXACT=1: every face through the exact (sqrtf) Gabor instance (tests)
  int channel_streams = 1;  // streams the channel stage is spread over (FFD_CHANNEL_STREAMS; 2-4 measured no gain)
  int host_chunk = 1024;    // faces per upload chunk of the host-buffer API (FFD_HOST_CHUNK)
  hipStream_t copy_stream = nullptr;  // H2D of the host-buffer API's images
  hipEvent_t copy_done = nullptr;
  int small_batch = 64;     // chunks of at most this many faces spread the channel stage over 6 streams (FFD_SMALL_BATCH)
  // traversal tuning: patch block edge G (a workgroup walks all trees of a G x G block of patches
  // over an LDS copy of the block's integral window) and the persistent workgroups (one per CU).
  // Overridable with FFD_TRAV_G_{HP,FFD} / FFD_TRAV_WG / FFD_CHUNK / FFD_STREAMS.
  TravShape trav_g_hp{5, 4}, trav_g_mp{5, 5};
  int trav_wg = 256;

  // model parameters
  int face_size = 125, patch = 31, hp_trees = 0, n_forests = 0, ntrees_per_forest = 0;
  int64_t hp_leaves = 0, mp_leaves = 0;
  std::vector<int64_t> hp_tree_leaf_off, mp_tree_leaf_off;  // per tree: first leaf ordinal (+ the total at the end)

  // device model
  DevBuf gabor_coef, hp_nodes, hp_roots, hp_sizes, hp_m, mp_nodes, mp_roots, mp_sizes, mp_rec;
  DevBuf hp_pairs, mp_pairs;         // pair records for k_traverse (ffd_device.hpp "pair records")
  DevBuf hp_proots, mp_proots;       // per tree: index of its root pair
  DevBuf hp_far, mp_far;             // per pair: far offset of child 1's children (when > 65535)
  DevBuf hp_tops, mp_tops, hp_topi, mp_topi;  // per tree: heap-ordered top pair records + their indices
  int trav_top_max = TOP_CAP;        // tree-top entries staged per tree at most (FFD_TRAV_TOPMAX)
  std::vector<uint4> hp_nodes_h, mp_nodes_h;  // host copies until the walk nodes are built
  std::vector<int32_t> hp_roots_h, mp_roots_h;
  bool vote_rec_compact = false;     // 32-B vote records (else 64-B), see load_model
  int vote_bias_x = 0, vote_bias_y = 0;
  ffd_host::VoteRange vote_range;    // the offsets those records can add (FaceDesc::wide)
  bool force_wide = false;           // FFD_VOTES_WIDE=1: every face through the wide vote path (tests)
  std::string model_path;            // the FFDMODEL file (re-read for option-dependent tables)

  // Option-dependent leaf tables (head-pose values m, FFD vote records) for per-call estimator
  // options that differ from desc's (the static estimateHeadPose / estimateFacialFeatures take their
  // options per call, FaceForest.hpp:97-115), built on first use from the model's leaf payloads.
  struct AltTables {
    bool hp_ok = false, mp_ok = false;
    ffd_headpose_option hp{};
    ffd_multipart_option mp{};
    DevBuf hp_m, mp_rec;
    bool compact = false;
    int bias_x = 0, bias_y = 0;
    ffd_host::VoteRange range;
  } alt;
  std::shared_ptr<ffd::ModelFile> leaf_model;  // leaf payload arrays (hp.leaf_*, mp.leaf_*), lazily
  const ffd::ModelFile& leaf_arrays();

  // Haar face detector (ffd_detect.cpp): the model's cascade, when it has one
  bool have_haar = false;
  int haar_ww = 0, haar_wh = 0, haar_stages = 0;
  DevBuf haar_weak, haar_stage;
  int haar_order_free = 0;  // every stage's leaf sum is exact in any order (ffd_detect.cpp load_cascade)
  int haar_nweak = 0;  // weak classifiers per ystep table (haar_weak holds two)
  DevBuf det_frames, det_levels, det_gray, det_scaled, det_sum, det_sq, det_res, det_cand, det_ncand, det_rowcnt, det_clsrect,
      det_clssum, det_boxes, det_packed, det_label;
  int n_cu = 256;  // compute units of the device (survivor-pass grids)

  std::vector<std::unique_ptr<Workspace>> ws;
  DevBuf images, out, scratch_a, scratch_b, scratch_c;  // host-API staging (ws[0] stream)
  // image samples (ffd_sample_*): pinned host buffers the evaluation kernel writes its leaf ordinals to,
  // and the staging of long patch lists
  struct Pinned {
    void* p = nullptr;
    size_t n = 0;
    void* ensure(size_t bytes) {
      if (bytes <= n) return p;
      if (p) (void)hipHostFree(p);
      p = nullptr;
      n = 0;
      HIP_CHECK(hipHostMalloc(&p, std::max<size_t>(bytes, 4096), hipHostMallocDefault));
      n = std::max<size_t>(bytes, 4096);
      return p;
    }
    ~Pinned() { if (p) (void)hipHostFree(p); }
  } pin_leaf, pin_patch;
  DevBuf sample_patches;
  int last_ws = -1;
  // live image samples (ffd_sample_*): a sample destroyed after its engine must not touch the engine, so the
  // engine frees the samples' device planes when it goes and marks them orphaned (ffd_engine_destroy)
  std::mutex samples_mu;
  std::unordered_set<ffd_sample*> samples;
  void track_sample(ffd_sample* s) {
    std::lock_guard<std::mutex> g(samples_mu);
    samples.insert(s);
  }
  void untrack_sample(ffd_sample* s) {
    std::lock_guard<std::mutex> g(samples_mu);
    samples.erase(s);
  }
  void orphan_samples();  // ffd_engine.cpp

  hipStream_t main_stream() const { return ws[0]->stream; }

  // stage profiler (hipEvents around each launch, on the launching stream)
  struct Pending { int stage; hipEvent_t a, b; };
  bool profiling = false;
  std::vector<hipEvent_t> event_pool;
  std::vector<Pending> pending;
  double stage_ms[FFD_NUM_STAGES] = {0};
  int64_t stage_n[FFD_NUM_STAGES] = {0};

  hipEvent_t get_event() {
    if (!event_pool.empty()) { hipEvent_t e = event_pool.back(); event_pool.pop_back(); return e; }
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));
    return e;
  }
  template <class F> void stage(int id, hipStream_t s, F&& fn) {
    if (!profiling) { fn(); return; }
    Pending p{id, get_event(), get_event()};
    HIP_CHECK(hipEventRecord(p.a, s));
    fn();
    HIP_CHECK(hipEventRecord(p.b, s));
    pending.push_back(p);
  }
  void sync_all() {  // (a stream with nothing queued answers the query at once: no wait)
    auto idle = [](hipStream_t s) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipErrorNotReady) return false;
      HIP_CHECK(q);
      return true;
    };
    if (copy_stream && !idle(copy_stream)) HIP_CHECK(hipStreamSynchronize(copy_stream));
    for (auto& w : ws) {
      for (auto f : w->fork)
        if (!idle(f)) HIP_CHECK(hipStreamSynchronize(f));
      if (!idle(w->stream)) HIP_CHECK(hipStreamSynchronize(w->stream));
    }
  }
  void resolve() {
    if (pending.empty()) return;
    sync_all();
    for (auto& p : pending) {
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, p.a, p.b));
      stage_ms[p.stage] += ms;
      stage_n[p.stage] += 1;
      event_pool.push_back(p.a);
      event_pool.push_back(p.b);
    }
    pending.clear();
  }

  // Pinned staging of the per-chunk face descriptors: a ring of slots, each reused only after the
  // copy that last read it has run (its event), so the host can refill descriptors for the next
  // chunk while earlier copies are still queued.
  struct PinnedSlot {
    void* p = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    bool used = false;
  };
  PinnedSlot desc_pin[8];
  int desc_pin_next = 0;
  // every slot's event and a first pinned buffer at engine creation: a slot's first use otherwise pays a
  // hipHostMalloc (≈ 50 µs) inside a call (the first eight calls of a process: evaluate_mt trace)
  void warm_descriptor_slots() {
    for (auto& s : desc_pin) {
      if (!s.ev) HIP_CHECK(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
      if (!s.p) {
        HIP_CHECK(hipHostMalloc(&s.p, 64 * sizeof(FaceDesc), hipHostMallocDefault));
        s.cap = 64 * sizeof(FaceDesc);
      }
    }
  }
  void upload_descriptors(DevBuf& dst, const std::vector<FaceDesc>& fds, hipStream_t st) {
    const size_t bytes = fds.size() * sizeof(FaceDesc);
    dst.ensure(bytes);
    upload_pinned(dst.p, fds.data(), bytes, st);
  }
  // a small host -> device copy through the pinned slots (a pageable source is staged by the runtime on
  // the calling thread)
  void upload_pinned(void* dst, const void* src, size_t bytes, hipStream_t st) {
    if (!bytes) return;
    PinnedSlot& s = desc_pin[desc_pin_next++ & 7];
    if (!s.ev) HIP_CHECK(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
    if (s.used) HIP_CHECK(hipEventSynchronize(s.ev));
    if (s.cap < bytes) {
      if (s.p) HIP_CHECK(hipHostFree(s.p));
      s.p = nullptr;
      s.cap = 0;
      HIP_CHECK(hipHostMalloc(&s.p, bytes, hipHostMallocDefault));
      s.cap = bytes;
    }
    std::memcpy(s.p, src, bytes);
    HIP_CHECK(hipMemcpyAsync(dst, s.p, bytes, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipEventRecord(s.ev, st));
    s.used = true;
  }

  ~ffd_engine() {
    for (auto& s : desc_pin) {
      if (s.used) (void)hipEventSynchronize(s.ev);
      if (s.ev) (void)hipEventDestroy(s.ev);
      if (s.p) (void)hipHostFree(s.p);
    }
    for (auto& p : pending) { event_pool.push_back(p.a); event_pool.push_back(p.b); }
    for (auto e : event_pool) (void)hipEventDestroy(e);
    if (copy_done) (void)hipEventDestroy(copy_done);
    if (copy_stream) (void)hipStreamDestroy(copy_stream);
  }

  Geometry geometry(int bw, int bh) const {
    Geometry g;
    if (bw <= 0 || bh <= 0) return g;
    g.scale = (float)face_size / (float)bw;  // FaceForest.cpp:202
    g.W = (int)((float)bw * g.scale);        // cv::Size(cols*scale, rows*scale) truncation
    g.H = (int)((float)bh * g.scale);
    auto cnt = [&](int extent, int step) {
      int n = 0;
      for (int x = 0; x < extent - patch; x += step) n++;
      return n;
    };
    g.nhx = cnt(g.W, desc.hp_option.step_size);
    g.nhy = cnt(g.H, desc.hp_option.step_size);
    g.nmx = cnt(g.W, desc.mp_option.step_size);
    g.nmy = cnt(g.H, mp_step_y());
    return g;
  }

  void load_model(const std::string& path);
  void load_cascade(const ffd::ModelFile& m);  // ffd_detect.cpp
  void build_gabor();
  // FFD patch-grid step along y: the reference has one step for both axes (step_size_y == 0)
  int mp_step_y() const { return desc.mp_option.step_size_y > 0 ? desc.mp_option.step_size_y : desc.mp_option.step_size; }
  // Fit the traversal window into the CU's 160 KB of LDS (and the staging registers), shrinking
  // the patch block if needed, and raise the kernels' dynamic-LDS limit.
  // The preferred patch-block shape, else the shapes below it (instantiated in ffd_kernels.hip)
  // whose window fits the LDS at these grid steps.
  static TravShape fit_shape(TravShape g, bool hp, int step, int step_y) {
    const TravShape cands[] = {g, {5, 5}, {5, 4}, {4, 4}, {3, 3}};
    for (const TravShape& c : cands)
      if (c.gx * c.gy <= g.gx * g.gy && traverse_shape_supported(c, hp) &&
          traverse_window_fits(c, hp, step, step_y, TRAV_LDS_CAP))
        return c;
    throw std::runtime_error("traversal window does not fit in LDS (step size too large)");
  }
  void check_traverse_lds() {
    const int cap = TRAV_LDS_CAP;
    trav_g_hp = fit_shape(trav_g_hp, true, desc.hp_option.step_size, desc.hp_option.step_size);
    trav_g_mp = fit_shape(trav_g_mp, false, desc.mp_option.step_size, mp_step_y());
    auto pairs = [&](std::vector<uint4>& h, std::vector<int32_t>& roots, DevBuf& d, DevBuf& droots, DevBuf& dfar,
                     DevBuf& dtops, DevBuf& dtopi) {
      std::vector<uint4> pr, tops;
      std::vector<int32_t> rp;
      std::vector<uint32_t> far, topi;
      ffd_host::build_pair_records(h, roots, pr, rp, far);
      ffd_host::build_tree_tops(pr, rp, far, tops, topi);
      upload(d, pr, main_stream());
      upload(droots, rp, main_stream());
      upload(dfar, far, main_stream());
      upload(dtops, tops, main_stream());
      upload(dtopi, topi, main_stream());
      HIP_CHECK(hipStreamSynchronize(main_stream()));
      std::vector<uint4>().swap(h);
      std::vector<int32_t>().swap(roots);
    };
    pairs(hp_nodes_h, hp_roots_h, hp_pairs, hp_proots, hp_far, hp_tops, hp_topi);
    pairs(mp_nodes_h, mp_roots_h, mp_pairs, mp_proots, mp_far, mp_tops, mp_topi);
    HIP_CHECK(set_traverse_lds_limit(cap));
    HIP_CHECK(set_gabor_lds_limit(96 * 1024));  // padded u8 face of up to MAX_FACE_H rows
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, device));
    if (!std::getenv("FFD_TRAV_WG")) trav_wg = std::max(8, prop.multiProcessorCount);
    n_cu = std::max(1, prop.multiProcessorCount);
  }
  void run_chunk(Workspace& w, const uint8_t* d_images, FaceOut* d_out);
  void analyze(const uint8_t* d_images, const std::vector<FaceDesc>& all, FaceOut* d_out);
};

namespace ffd_host {
// option-dependent leaf tables (ffd_engine.cpp)
std::vector<float> hp_leaf_values(const ffd::ModelFile& m, const ffd_headpose_option& o);
struct VoteTable {
  std::vector<uint32_t> rec;
  bool compact = false;
  int bias_x = 0, bias_y = 0;
  VoteRange range;
};
VoteTable mp_vote_records(const ffd::ModelFile& m, const ffd_multipart_option& o);
// status + message helpers shared by the C entry points
ffd_status fail(ffd_engine* e, ffd_status s, const std::string& msg);
// analyzeFace over host images: upload, descriptors, pipeline; results left in d_out (device)
ffd_status analyze_host(ffd_engine* e, const ffd_image* imgs, int32_t n_img, const ffd_rect* boxes,
                        const int32_t* box_img, int32_t n_faces, void* d_out);
// per-face descriptor of a box on an image (ffd_engine.cpp); returns the face's status
ffd_status make_desc(const ffd_engine* e, int64_t img_off, int iw, int ih, int stride, const ffd_rect& b, FaceDesc& f);
// a Haar cascade XML (OpenCV format) as the FFDMODEL "haar.*" arrays (ffd_convert.cpp); throws on failure
void cascade_arrays(const std::string& xml, ffd::ModelFile& m);
// the engine's per-rank RCCL communicator, if it joined one (ffd_group.cpp)
void release_comm(const ffd_engine* e);
}  // namespace ffd_host
