// ffd_group.cpp — multi-GPU entry points of libffd.so (include/ffd.h "multi-device").
//
// Faces are independent: the reference loops them (src/FaceForest.cpp:175-180) and shares only the
// read-only forests.  So every device holds its own copy of the model (one ffd_engine each), owns a
// contiguous block of ceil(N / G) faces, runs the whole path on it with no data-path exchange, and
// the ffd_face records are gathered to one device in ONE RCCL gather over xGMI (~112 B per face).
//   ffd_group_*            one process driving G devices (ncclCommInitAll);
//   ffd_comm_id / ffd_engine_join / ffd_gather_faces
//                          one process per device (ncclCommInitRank; the caller shares the 128-byte
//                          id the way its launcher shares anything, e.g. an MPI / torch broadcast).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ffd_engine_impl.hpp"

namespace {

using namespace ffd_host;

struct NcclError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define NCCL_CHECK(expr)                                                                    \
  do {                                                                                      \
    ncclResult_t r_ = (expr);                                                               \
    if (r_ != ncclSuccess) throw NcclError(std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

constexpr size_t REC = sizeof(ffd_face);

void shard(int n, int world, int rank, int& lo, int& hi) {
  const int per = (n + world - 1) / world;
  lo = std::min(n, rank * per);
  hi = std::min(n, lo + per);
}

thread_local std::string g_group_err;

// Runs fn(d) for every device d < G, device 0 on the calling thread and the others on threads of their own:
// a device's shard reaches it by pageable host copies that the runtime stages on the calling thread, so one
// host thread per device lets the uploads (and the launches) of all devices proceed at once.  Returns the
// per-device status; a device whose fn throws gets FFD_ERR_DEVICE / FFD_ERR_INTERNAL and its message.
template <class F> std::vector<ffd_status> for_each_device(int G, std::vector<std::string>& errs, F&& fn) {
  std::vector<ffd_status> st(G, FFD_OK);
  errs.assign(G, std::string());
  auto run = [&](int d) {
    try {
      st[d] = fn(d);
    } catch (const HipError& x) {
      st[d] = FFD_ERR_DEVICE;
      errs[d] = x.what();
    } catch (const std::exception& x) {
      st[d] = FFD_ERR_INTERNAL;
      errs[d] = x.what();
    }
  };
  std::vector<std::thread> th;
  for (int d = 1; d < G; d++) th.emplace_back(run, d);
  run(0);
  for (auto& t : th) t.join();
  return st;
}

}  // namespace

struct ffd_group {
  std::string err;
  std::vector<int> devices;
  std::vector<ffd_engine*> engines;
  std::vector<ncclComm_t> comms;
  std::vector<std::unique_ptr<DevBuf>> local;  // per device: its shard's records (padded to ceil(N/G))
  DevBuf gathered;                             // on devices[0]: G * ceil(N/G) records
  ~ffd_group() {
    for (size_t i = 0; i < comms.size(); i++)
      if (comms[i]) (void)ncclCommDestroy(comms[i]);
    for (size_t i = 0; i < local.size(); i++) {
      (void)hipSetDevice(devices[i]);
      local[i].reset();
    }
    if (!devices.empty()) (void)hipSetDevice(devices[0]);
    for (auto* e : engines) ffd_engine_destroy(e);
  }
};

namespace {

template <class F> ffd_status group_guarded(ffd_group* g, F&& fn) {
  if (!g) return FFD_ERR_INVALID_ARGUMENT;
  try {
    return fn();
  } catch (const NcclError& x) {
    g->err = x.what();
    return FFD_ERR_DEVICE;
  } catch (const HipError& x) {
    g->err = x.what();
    return FFD_ERR_DEVICE;
  } catch (const std::exception& x) {
    g->err = x.what();
    return FFD_ERR_INTERNAL;
  }
}

// per-rank communicators of engines that joined one (ffd_engine_join), released with the engine.
// Several engines of one process may join, gather and be destroyed on different threads: every map
// access holds comm_mu, which is never held across ncclCommInitRank (that call blocks until all the
// communicator's ranks have joined, possibly from other threads of this process).
std::mutex comm_mu;
std::map<const ffd_engine*, ncclComm_t>& rank_comms() {
  static std::map<const ffd_engine*, ncclComm_t> m;
  return m;
}
ncclComm_t find_comm(const ffd_engine* e) {
  std::lock_guard<std::mutex> lk(comm_mu);
  auto it = rank_comms().find(e);
  return it == rank_comms().end() ? nullptr : it->second;
}

}  // namespace

void ffd_host::release_comm(const ffd_engine* e) {
  ncclComm_t c = nullptr;
  {
    std::lock_guard<std::mutex> lk(comm_mu);
    auto& m = rank_comms();
    auto it = m.find(e);
    if (it == m.end()) return;
    c = it->second;
    m.erase(it);
  }
  (void)ncclCommDestroy(c);
}

extern "C" {

ffd_status ffd_group_create(const ffd_engine_desc* desc, const int32_t* devices, int32_t n_devices, ffd_group** out) {
  if (!out) return FFD_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  if (!desc || !devices || n_devices < 1) {
    g_group_err = "desc / devices missing";
    return FFD_ERR_INVALID_ARGUMENT;
  }
  std::unique_ptr<ffd_group> g(new ffd_group());
  g->devices.assign(devices, devices + n_devices);
  for (int i = 0; i < n_devices; i++) {
    ffd_engine_desc d = *desc;
    d.device = devices[i];
    ffd_engine* e = nullptr;
    const ffd_status st = ffd_engine_create(&d, &e);
    if (st != FFD_OK) {
      g_group_err = std::string("device ") + std::to_string(devices[i]) + ": " + ffd_last_error(nullptr);
      return st;
    }
    g->engines.push_back(e);
    g->local.emplace_back(new DevBuf());
  }
  g->comms.assign(n_devices, nullptr);
  const ncclResult_t r = ncclCommInitAll(g->comms.data(), n_devices, g->devices.data());
  if (r != ncclSuccess) {
    g->comms.clear();
    g_group_err = std::string("ncclCommInitAll: ") + ncclGetErrorString(r);
    return FFD_ERR_DEVICE;
  }
  *out = g.release();
  return FFD_OK;
}

void ffd_group_destroy(ffd_group* g) { delete g; }

const char* ffd_group_last_error(const ffd_group* g) { return g ? g->err.c_str() : g_group_err.c_str(); }

int32_t ffd_group_size(const ffd_group* g) { return g ? (int32_t)g->engines.size() : 0; }

ffd_engine* ffd_group_engine(ffd_group* g, int32_t i) {
  return (g && i >= 0 && i < (int32_t)g->engines.size()) ? g->engines[i] : nullptr;
}

ffd_status ffd_group_analyze_faces(ffd_group* g, const ffd_image* imgs, int32_t n_img, const ffd_rect* boxes,
                                   const int32_t* box_img, int32_t n_faces, ffd_face* out) {
  return group_guarded(g, [&]() -> ffd_status {
    if (n_faces < 0 || (n_faces > 0 && (!imgs || !boxes || !out)) || n_img < 0) {
      g->err = "bad arguments";
      return FFD_ERR_INVALID_ARGUMENT;
    }
    if (!box_img && n_img != n_faces) {
      g->err = "box_img NULL requires n_img == n_faces";
      return FFD_ERR_INVALID_ARGUMENT;
    }
    if (n_faces == 0) return FFD_OK;
    const int G = (int)g->engines.size(), per = (n_faces + G - 1) / G;
    for (int i = 0; i < n_faces; i++) {
      const int k = box_img ? box_img[i] : i;
      if (k < 0 || k >= n_img) {
        g->err = "box_img out of range";
        return FFD_ERR_INVALID_ARGUMENT;
      }
    }
    // every device, on a host thread of its own: its contiguous face block, with only the images those faces
    // reference (the engines are independent objects; each thread touches only its own)
    std::vector<std::string> errs;
    const std::vector<ffd_status> sts = for_each_device(G, errs, [&](int d) -> ffd_status {
      int lo, hi;
      shard(n_faces, G, d, lo, hi);
      HIP_CHECK(hipSetDevice(g->devices[d]));
      g->local[d]->ensure((size_t)per * REC);
      HIP_CHECK(hipMemsetAsync(g->local[d]->p, 0, (size_t)per * REC, (hipStream_t)ffd_stream(g->engines[d])));
      if (hi <= lo) return FFD_OK;
      std::vector<int32_t> remap(n_img, -1), sub_box_img;
      std::vector<ffd_image> sub_imgs;
      for (int i = lo; i < hi; i++) {
        const int k = box_img ? box_img[i] : i;
        if (remap[k] < 0) {
          remap[k] = (int32_t)sub_imgs.size();
          sub_imgs.push_back(imgs[k]);
        }
        sub_box_img.push_back(remap[k]);
      }
      return analyze_host(g->engines[d], sub_imgs.data(), (int32_t)sub_imgs.size(), boxes + lo, sub_box_img.data(),
                          hi - lo, g->local[d]->p);
    });
    for (int d = 0; d < G; d++)
      if (sts[d] != FFD_OK) {
        g->err = std::string("device ") + std::to_string(g->devices[d]) + ": " +
                 (errs[d].empty() ? std::string(ffd_last_error(g->engines[d])) : errs[d]);
        return sts[d];
      }
    // one gather of every device's (padded) records to devices[0], on each engine's stream
    HIP_CHECK(hipSetDevice(g->devices[0]));
    g->gathered.ensure((size_t)G * per * REC);
    NCCL_CHECK(ncclGroupStart());
    for (int d = 0; d < G; d++)
      NCCL_CHECK(ncclGather(g->local[d]->p, d == 0 ? g->gathered.p : nullptr, (size_t)per * REC, ncclUint8, 0,
                            g->comms[d], (hipStream_t)ffd_stream(g->engines[d])));
    NCCL_CHECK(ncclGroupEnd());
    HIP_CHECK(hipSetDevice(g->devices[0]));
    const hipStream_t s0 = (hipStream_t)ffd_stream(g->engines[0]);
    for (int d = 0; d < G; d++) {
      int lo, hi;
      shard(n_faces, G, d, lo, hi);
      if (hi > lo)
        HIP_CHECK(hipMemcpyAsync(out + lo, g->gathered.as<uint8_t>() + (size_t)d * per * REC, (size_t)(hi - lo) * REC,
                                 hipMemcpyDeviceToHost, s0));
    }
    HIP_CHECK(hipStreamSynchronize(s0));
    for (int d = 1; d < G; d++) {
      HIP_CHECK(hipSetDevice(g->devices[d]));
      HIP_CHECK(hipStreamSynchronize((hipStream_t)ffd_stream(g->engines[d])));
    }
    return FFD_OK;
  });
}

ffd_status ffd_group_debug_overlap(int32_t n, int32_t ms, double* wall_ms) {
  if (n < 1 || ms < 0 || !wall_ms) return FFD_ERR_INVALID_ARGUMENT;
  std::vector<std::string> errs;
  const auto t0 = std::chrono::steady_clock::now();
  for_each_device(n, errs, [&](int) -> ffd_status {
    std::this_thread::sleep_for(std::chrono::milliseconds(ms));
    return FFD_OK;
  });
  *wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return FFD_OK;
}

ffd_status ffd_comm_id(uint8_t* id) {
  if (!id) return FFD_ERR_INVALID_ARGUMENT;
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) {
    g_group_err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
    return FFD_ERR_DEVICE;
  }
  static_assert(sizeof(u) == FFD_COMM_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id, &u, sizeof(u));
  return FFD_OK;
}

ffd_status ffd_engine_join(ffd_engine* e, const uint8_t* id, int32_t n_ranks, int32_t rank) {
  if (!e || !id || n_ranks < 1 || rank < 0 || rank >= n_ranks) return FFD_ERR_INVALID_ARGUMENT;
  try {
    HIP_CHECK(hipSetDevice(e->device));
    release_comm(e);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    NCCL_CHECK(ncclCommInitRank(&c, n_ranks, u, rank));
    std::lock_guard<std::mutex> lk(comm_mu);
    rank_comms()[e] = c;
    return FFD_OK;
  } catch (const std::exception& x) {
    return fail(e, FFD_ERR_DEVICE, x.what());
  }
}

ffd_status ffd_gather_faces(ffd_engine* e, const void* d_local, int32_t n_per_rank, void* d_root, int32_t root) {
  if (!e || (n_per_rank > 0 && !d_local) || n_per_rank < 0) return FFD_ERR_INVALID_ARGUMENT;
  try {
    const ncclComm_t c = find_comm(e);
    if (!c) return fail(e, FFD_ERR_NOT_INITIALIZED, "engine has not joined a communicator");
    HIP_CHECK(hipSetDevice(e->device));
    int rank = 0;
    NCCL_CHECK(ncclCommUserRank(c, &rank));
    if (rank == root && !d_root) return fail(e, FFD_ERR_INVALID_ARGUMENT, "root needs a receive buffer");
    NCCL_CHECK(ncclGather(d_local, rank == root ? d_root : nullptr, (size_t)n_per_rank * REC, ncclUint8, root,
                          c, e->main_stream()));
    return FFD_OK;
  } catch (const std::exception& x) {
    return fail(e, FFD_ERR_DEVICE, x.what());
  }
}

ffd_status ffd_engine_comm_info(ffd_engine* e, int32_t* n_ranks, int32_t* rank) {
  if (!e || !n_ranks || !rank) return FFD_ERR_INVALID_ARGUMENT;
  try {
    const ncclComm_t c = find_comm(e);
    if (!c) return fail(e, FFD_ERR_NOT_INITIALIZED, "engine has not joined a communicator");
    int n = 0, r = 0;
    NCCL_CHECK(ncclCommCount(c, &n));
    NCCL_CHECK(ncclCommUserRank(c, &r));
    *n_ranks = n;
    *rank = r;
    return FFD_OK;
  } catch (const std::exception& x) {
    return fail(e, FFD_ERR_DEVICE, x.what());
  }
}

}  // extern "C"
