"""Benchmark: faces/sec of FaceForest::analyzeFace on the pretrained FFD forest (BASELINE.json).

Workload (config C2, BASELINE.json configs[1]): per GPU, a batch of 4,096 synthetic 150x150 BGR
face crops (face_alignment_cvpr_2012_amd/synthetic.py, seed 2012 + rank), analyzeFace(crop,
Rect(0,0,150,150)) each -> 125x125 face, 576 head-pose + 1,024 FFD patches, 15 + 20 trees.
A step = one full pass of the hot path over the batch: gray/resize, 38 integral channels,
head-pose forest, tree selection, FFD forest, votes, MeanShift.  Inputs are resident in HBM when
the timed region starts; outputs stay in HBM (for N > 1 they are gathered to rank 0 with an
RCCL gather over xGMI inside the step).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4|c5]
N > 1: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) WORLD_SIZE must equal N;
run directly, bench.py starts the N ranks itself (torch.distributed.run as a child process, before
anything touches the GPU) and exits with its status.  Rank 0 prints ONE JSON line.
--dry-run: the launcher and the record gather without a GPU (gloo, synthetic records; tests).
"""
import argparse
import glob
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3     # MI355X FP32 vector = FP32 matrix peak (no dense MFMA work here)
CROP = 150


def gabor_flops_per_pixel(w, face_w=125):
    """FLOPs the restated Gabor correlation executes per output pixel for the 7 orientations of
    one scale.  7x7: OpenCV's direct filter, mul + add per tap for re and im.
    >= 9x9 (separable definition, include/ffd_gabor.h): V pass per padded column ((W + 2R) / W
    of the pixels): per folded pair S, D + 9 FMAs, centre 9 FMAs; H pass per tap 25 FMAs
    (DC, mu 0 and mu 4 one pair each, the other four orientations two pairs each), DC term 7 FMAs.
    + magnitude (2 mul, add, sqrt) per orientation."""
    if w == 7:
        core = 49 * 7 * 2 * 2
    else:
        r = (w - 1) // 2
        v = (r * (2 + 9 * 2) + 9 * 2) * (face_w + 2 * r) / face_w
        core = v + w * 25 * 2 + 7 * 2
    return core + 7 * 4


# profiler stage -> kernel name prefix in rocprofv3 traces (for the PMC traffic lookup)
STAGE_KERNELS = {
    "gray_resize": "ffd::k_gray_resize", "gabor_25x25": "void ffd::k_gabor_sep<25, false>",
    "gabor_19x19": "void ffd::k_gabor_sep<19, false>", "gabor_13x13": "void ffd::k_gabor_sep<13, false>",
    "gabor_9x9": "void ffd::k_gabor_sep<9, false>", "gabor_7x7": "void ffd::k_gabor7<false>",
    "integral_channels": "ffd::k_integral", "headpose_traverse": "void ffd::k_traverse<true",
    "headpose_reduce_select": "ffd::k_hp_pose", "ffd_traverse": "void ffd::k_traverse<false",
    "votes": "ffd::k_votes", "meanshift": "ffd::k_meanshift",
}


SOURCE_FILES = ("face_alignment_cvpr_2012_amd/csrc/ffd_kernels.hip", "face_alignment_cvpr_2012_amd/csrc/ffd_engine.cpp",
                "face_alignment_cvpr_2012_amd/csrc/ffd_device.hpp", "face_alignment_cvpr_2012_amd/csrc/ffd_kernels.hpp",
                "include/ffd_numerics.h", "include/ffd_gabor.h")


def source_digest():
    """sha256 (16 hex) of the kernel and engine sources: ties a PMC summary to the code it measured
    (the GPU box gets no .git, so the commit id is not available there)."""
    h = hashlib.sha256()
    for f in SOURCE_FILES:
        with open(os.path.join(REPO, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def measured_traffic(stage, faces_per_launch, workload="c2", key="traffic_bytes"):
    """HBM bytes per launch of `stage`'s kernel from the committed PMC summary of THIS source tree
    (profiles/<round>/traffic.json with a matching source_digest, written by tools/pmc_traffic.py
    from tools/profile_round.sh's FETCH_SIZE / WRITE_SIZE passes over the same workload), or None
    (no summary was collected for the code being measured)."""
    import glob
    digest = source_digest()
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*", "traffic.json")), reverse=True):
        try:
            doc = json.load(open(path))
        except (OSError, ValueError):
            continue
        if doc.get("source_digest") != digest or doc.get("workload", "c2") != workload:
            continue
        if doc.get("faces_per_launch", 4096) != faces_per_launch:
            continue
        pre = STAGE_KERNELS.get(stage)
        for name, v in doc.get("kernels", {}).items():
            if pre and name.startswith(pre) and v.get(key):
                return v[key]
    return None


def gather_figure(stage, avg_ms, faces_per_launch, n_cu):
    """roofline.gather (VERDICT r5 "next" #3): the traversal's record gathers priced at the gather probe's cost, as a
    fraction of the kernel's measured time.  Gathers per face (wave-level deep-loop gathers x their active lanes) come
    from the walk statistics tools/walk_locality.py computes on C2 faces with k_traverse's lane mapping
    (profiles/*/walk_locality.json, newest); the cost per gathered lane is tools/td_probe.hip's 16-B gather with 64
    distinct 128-B lines per wave-instruction from a 2 MB (L2-resident) table (profiles/r5a/td_probe.json).  1.0 =
    the kernel's whole time is its gathers' vector-memory data-path time at that rate (the walk-only probe measured
    TD busy at that level)."""
    kind = {"ffd_traverse": "ffd", "headpose_traverse": "hp"}.get(stage)
    if kind is None:
        return None
    walk = probe = None
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*", "walk_locality.json")), reverse=True):
        walk = json.load(open(path))
        walk_src = os.path.relpath(path, REPO)
        break
    probe_path = os.path.join(REPO, "profiles", "r5a", "td_probe.json")
    if os.path.exists(probe_path):
        for line in open(probe_path):
            r = json.loads(line)
            if r["table_kb"] == 2048 and r["bytes"] == 16 and r["active"] == 64 and r["lines"] == 64:
                probe = r
    if walk is None or probe is None or kind not in walk:
        return None
    w = walk[kind]["dfs"]
    lanes = w["lane_gathers_per_face"] * faces_per_launch
    gather_ms = lanes / n_cu * probe["ns_per_lane"] / 1e6
    return {"frac": round(gather_ms / avg_ms, 4), "gather_ms": round(gather_ms, 4), "kernel_ms": round(avg_ms, 4),
            "lane_gathers_per_launch": int(lanes), "lines_per_instr": round(w["lines_per_instr"], 2),
            "ns_per_lane": probe["ns_per_lane"], "cus": n_cu, "walk_stats": walk_src,
            "probe": "profiles/r5a/td_probe.json (16 B, 64 lines, 2 MB table)"}


def stage_work(stage, n_faces, W=125, H=125, n_hp=576, n_mp=1024, trees=20):
    """Algorithmic work of one launch of `stage` over n_faces: (amount, unit, bound).
    Integral channels are stored as u16 (integral mod 2^16, DESIGN.md §Data layout)."""
    chan_bytes = 38 * (H + 1) * (W + 1) * 2
    if stage.startswith("gabor_"):
        w = int(stage.split("_")[1].split("x")[0])
        return n_faces * W * H * gabor_flops_per_pixel(w, W) / 1e12, "TFLOP/s", "valu"
    if stage == "integral_channels":
        return n_faces * (35 * W * H * 4 + W * H + chan_bytes) / 1e9, "GB/s", "hbm"  # read mag+gray, write planes
    if stage == "headpose_traverse":
        return n_faces * (chan_bytes + n_hp * 15 * 4) / 1e9, "GB/s", "hbm"
    if stage == "ffd_traverse":
        return n_faces * (chan_bytes + n_mp * trees * 4) / 1e9, "GB/s", "hbm"
    if stage == "votes":  # leaf ids in, each (patch, tree) leaf's 32-B vote record gathered, votes out
        return n_faces * (n_mp * trees * (4 + 32) + 1700 * 10 * 8) / 1e9, "GB/s", "hbm"
    if stage == "meanshift":
        return n_faces * (1700 * 10 * 8 + 112) / 1e9, "GB/s", "hbm"
    if stage == "gray_resize":
        return n_faces * (CROP * CROP * 3 + W * H) / 1e9, "GB/s", "hbm"
    return n_faces * n_hp * 15 * 4 / 1e9, "GB/s", "hbm"


def host_cores():
    """Host threads this process may use: its CPU affinity, capped by OMP_NUM_THREADS (the GPU box
    sets it to the box's CPU share, 16 per GPU; nproc there shows the whole machine)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return max(1, min(avail, int(os.environ.get("OMP_NUM_THREADS", avail))))


def cpu_baseline(wl, n_budget_s=12.0):
    """Oracle (C++ restatement) timed on the host cores, on bounded samples (~n_budget_s seconds
    each) of the benchmarked workload's own faces:
      value          reference-shaped: faces sequential, per-face thread pools of `cores` threads
                     for the 35 Gabor, the head-pose and the FFD patch tasks (ThreadPool.hpp:24-64,
                     the reference's hardware_concurrency() pools sized to the cores available);
      faces_parallel labelled alternative: `cores` faces at once, one thread each."""
    import concurrent.futures as cf

    import oracle
    oracle.load_model(wl.model)
    oracle.set_steps(4, *wl.mp_steps)
    cores = host_cores()
    face = lambda k: wl.face(k % wl.n)  # noqa: E731
    t0 = time.perf_counter()
    oracle.analyze_face(*face(0), threads=cores)
    one = time.perf_counter() - t0
    n = int(max(3, min(4 * wl.n, n_budget_s / max(one, 1e-3))))
    t0 = time.perf_counter()
    for k in range(1, n + 1):
        oracle.analyze_face(*face(k), threads=cores)
    dt = time.perf_counter() - t0
    # faces-parallel: ctypes releases the GIL, so `cores` Python threads run `cores` faces at once
    n_par = int(max(cores, min(4 * wl.n, n_budget_s * cores / max(one * cores, 1e-3))))
    with cf.ThreadPoolExecutor(cores) as ex:
        t0 = time.perf_counter()
        list(ex.map(lambda k: oracle.analyze_face(*face(k), threads=1), range(1, n_par + 1)))
        dt_par = time.perf_counter() - t0
    cpu = ""
    try:
        cpu = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return {"value": round(n / dt, 3), "unit": "faces/s", "cores": cores, "kind": "port",
            "sample": f"first {n} faces of the {wl.name} workload, analyzeFace each, reference-shaped per-face "
                      f"thread pools of {cores} threads, {dt:.1f} s; host {cpu}, nproc {os.cpu_count()}, "
                      f"affinity/OMP_NUM_THREADS share {cores}",
            "faces_parallel": {"value": round(n_par / dt_par, 3), "unit": "faces/s", "cores": cores,
                               "sample": f"{n_par} faces, {cores} at once (one thread each), {dt_par:.1f} s"}}


class Workload:
    """One GPU's share of a BASELINE.json config: host images, boxes, box -> image map."""

    def __init__(self, name, images, boxes, box_img, scaling, describe, total_faces, n_images=None,
                 model=None, mp_steps=(3, 3), seed=None, gt=None):
        self.name, self.images, self.box_img = name, images, box_img
        self.seed, self.gt = seed, gt  # generator seed; ground-truth landmarks (n, 10, 2) or None
        self.boxes = np.ascontiguousarray(np.asarray(boxes, np.int32).reshape(-1, 4))  # packed once
        self.scaling, self.describe, self.total_faces = scaling, describe, total_faces
        self.model = model or os.path.join(REPO, "model", "ffd_model.bin")
        self.mp_steps = mp_steps  # FFD patch-grid step (x, y)
        # images beyond the distinct ones repeat them cyclically (generation time; same work per image)
        self.n_images = n_images or len(images)

    @property
    def n(self):
        return len(self.boxes)

    def face(self, k):
        return self.images[self.box_img[k] % len(self.images)], tuple(int(v) for v in self.boxes[k])


def make_workload(name, rank, world, faces, frames):
    from face_alignment_cvpr_2012_amd.distributed import shard_bounds
    from face_alignment_cvpr_2012_amd.synthetic import crop_ground_truth, make_crops, make_frames
    if name == "c2":  # BASELINE configs[1]: 4096 crops per GPU (weak scaling)
        crops, _ = make_crops(faces, seed=2012 + rank)
        return Workload("c2", crops, [(0, 0, CROP, CROP)] * faces, np.arange(faces, dtype=np.int32), "weak",
                        f"C2: batch of {faces} pre-cropped 150x150 faces per GPU, pretrained config_ffd.txt forest "
                        "(20 trees/face of 5x20, depth<=20), head-pose forest 15 trees, 125x125 faces",
                        faces * world, seed=2012 + rank, gt=crop_ground_truth(faces, seed=2012 + rank))
    if name == "c3":  # configs[2]: 512 1080p frames dealt over the GPUs, 8 detectFace-enlarged boxes each
        lo, hi = shard_bounds(frames, world, rank)
        uniq = min(hi - lo, 64)
        fr, bx, _ = make_frames(uniq, seed=1080 + lo)
        boxes = [tuple(int(v) for v in bx[k % uniq, j]) for k in range(hi - lo) for j in range(bx.shape[1])]
        box_img = np.repeat(np.arange(hi - lo), bx.shape[1]).astype(np.int32)
        return Workload("c3", fr, boxes, box_img, "strong", n_images=hi - lo, describe=
                        f"C3: {frames} synthetic 1920x1080 frames sharded over the GPUs (64 distinct per GPU, "
                        "repeated), 8 faces each (paste boxes through the detectFace enlargement: 125 x ~148 faces), "
                        "pretrained forests", total_faces=frames * 8)
    if name == "c5":  # configs[4]: 64 faces/frame x 512 frames = 32768 crops over all GPUs (strong scaling)
        total = 64 * 512
        lo, hi = shard_bounds(total, world, rank)
        crops, _ = make_crops(hi - lo, seed=5000 + rank)
        return Workload("c5", crops, [(0, 0, CROP, CROP)] * (hi - lo), np.arange(hi - lo, dtype=np.int32), "strong",
                        "C5: 64 faces/frame x 512 frames = 32768 C2-style crops sharded over the GPUs, all 5 "
                        "pose-conditional FFD forests resident", total, seed=5000 + rank,
                        gt=crop_ground_truth(hi - lo, seed=5000 + rank))
    if name == "c4":  # configs[3]: synthetic 20 complete depth-20 trees, 4x patch density, 1 GPU
        path = synth_forest_path(20)
        crops, _ = make_crops(faces, seed=4000 + rank)
        return Workload("c4", crops, [(0, 0, CROP, CROP)] * faces, np.arange(faces, dtype=np.int32), "weak",
                        f"C4: {faces} C2-style crops per GPU on a synthetic forest of 20 complete depth-20 trees "
                        "(one forest for all pose bins), FFD grid step (2, 1): 4,418 patches x 20 walks per face",
                        faces * world, model=path, mp_steps=(2, 1))
    raise ValueError(name)


def synth_forest_path(depth):
    """C4's synthetic forest (face_alignment_cvpr_2012_amd/bin/ffd_synth_forest), generated once
    per box outside the repository (~3.7 GB at depth 20)."""
    import subprocess
    import tempfile
    path = os.path.join(tempfile.gettempdir(), f"ffd_c4_d{depth}.bin")
    if not os.path.exists(path):
        exe = os.path.join(REPO, "face_alignment_cvpr_2012_amd", "bin", "ffd_synth_forest")
        subprocess.run([exe, os.path.join(REPO, "model", "ffd_model.bin"), path + ".tmp", str(depth), "20", "4"],
                       check=True, stdout=subprocess.DEVNULL)
        os.replace(path + ".tmp", path)
    return path


C2_GOLDEN = os.path.join(REPO, "tests", "golden", "c2_golden.npz")


def landmark_error(wl, d_out, budget_s=10.0):
    """The metric's second half, 'mean landmark px error', outside the timed region: the rank's
    output records decoded and compared landmark by landmark (Euclidean px, eval_ffd.cpp:102-108's
    |gt - pred|) with the CPU restatement on identical inputs, and with the crops' annotated landmarks.
    C2 at its stated 4,096 faces (rank 0): EVERY face against the committed oracle goldens
    (tests/golden/c2_golden.npz); otherwise the oracle is run on the first faces for ~budget_s."""
    import face_alignment_cvpr_2012_amd as ffd
    faces = ffd.faces_from_records(d_out[: wl.n * ffd.FACE_RECORD_BYTES].cpu().numpy().tobytes())
    got = np.stack([f.ffd_cordinates for f in faces]).astype(np.float64)
    hp = np.array([f.headpose for f in faces], np.float32)
    out = {}
    g = np.load(C2_GOLDEN, allow_pickle=False) if os.path.exists(C2_GOLDEN) else None
    if wl.name == "c2" and g is not None and wl.n == g["points"].shape[0] and wl.seed == int(g["seed"]):
        ref, ref_hp, k = g["points"].astype(np.float64), g["headpose"], wl.n
        out["vs_cpu_source"] = f"all {k} faces vs tests/golden/c2_golden.npz (oracle, seed {wl.seed})"
    else:
        import concurrent.futures as cf

        import oracle
        oracle.load_model(wl.model)
        oracle.set_steps(4, *wl.mp_steps)
        t0, res = time.perf_counter(), []
        cores = host_cores()
        with cf.ThreadPoolExecutor(cores) as ex:
            while len(res) < wl.n and time.perf_counter() - t0 < budget_s:
                idx = range(len(res), min(wl.n, len(res) + cores))
                res += list(ex.map(lambda i: oracle.analyze_face(*wl.face(i), threads=1)[0], idx))
        k = len(res)
        ref = np.stack([r["points"] for r in res]).astype(np.float64)
        ref_hp = np.array([r["headpose"] for r in res], np.float32)
        out["vs_cpu_source"] = f"first {k} of {wl.n} faces vs the oracle run here"
    d = np.linalg.norm(got[:k] - ref, axis=2)
    out.update(vs_cpu_px=round(float(d.mean()), 6), vs_cpu_max_px=round(float(d.max()), 3), faces_checked=k,
               faces_identical=int(((d == 0).all(axis=1) & (hp[:k].view(np.uint32) == ref_hp.view(np.uint32))).sum()))
    if wl.gt is not None:
        e = np.linalg.norm(got - wl.gt[: wl.n], axis=2)
        out["vs_ground_truth_px"] = round(float(e.mean()), 4)
        out["ground_truth"] = "annotated landmarks of the source fixtures mapped into each crop (synthetic.crop_ground_truth)"
    return out


def host_inclusive(ff, wl, iw, ih, steps, warmup=1, chunks=4):
    """SURVEY.md §8(d)'s timing rule for the host API: batch in pinned host memory -> H2D -> the
    path -> D2H of the records, in `chunks` chunks whose H2D (own stream) overlaps the previous
    chunk's compute (engine stream).  C2-shaped workloads only (one image per face)."""
    import torch
    n, rec = wl.n, 112
    h_img = torch.from_numpy(np.ascontiguousarray(wl.images[:n])).pin_memory()
    d_img = torch.empty(h_img.shape, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(n * rec, dtype=torch.uint8, device="cuda")
    h_out = torch.empty(n * rec, dtype=torch.uint8).pin_memory()
    eng = torch.cuda.ExternalStream(ff.stream())
    copy = torch.cuda.Stream()
    bounds = [n * c // chunks for c in range(chunks + 1)]
    per_img = iw * ih * 3

    def run():
        for c in range(chunks):
            a, b = bounds[c], bounds[c + 1]
            if a == b:
                continue
            with torch.cuda.stream(copy):
                d_img[a:b].copy_(h_img[a:b], non_blocking=True)
                ev = copy.record_event()
            eng.wait_event(ev)
            ff.analyze_device(d_img[a].data_ptr(), per_img, iw, ih, iw * 3, b - a, wl.boxes[a:b],
                              np.arange(b - a, dtype=np.int32), d_out[a * rec].data_ptr())
            with torch.cuda.stream(eng):
                h_out[a * rec:b * rec].copy_(d_out[a * rec:b * rec], non_blocking=True)
        ff.synchronize()
        torch.cuda.synchronize()

    for _ in range(max(1, warmup)):
        run()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    dt = (time.perf_counter() - t0) / steps
    return {"value": round(n / dt, 1), "unit": "faces/s", "ms_per_step": round(dt * 1e3, 3), "chunks": chunks,
            "steps": steps, "warmup": max(1, warmup),
            "h2d_bytes": int(n * per_img), "note": "pinned host batch in, host records out; chunked H2D on its own "
                                                   "stream overlapping the previous chunk's compute"}


def cxx_host_path(wl, reps=5):
    """The C ABI's host-buffer path timed from C++ (examples/bench_host.cpp through include/FaceForest.hpp):
    FaceForest::analyzeFaces over the whole batch (pageable host crops in, host records out) and the
    reference's one-analyzeFace-per-call latency (eval_ffd.cpp:89).  Runs as a child process BEFORE this
    process touches the GPU (nothing here has initialised HIP yet)."""
    import tempfile
    exe = os.path.join(REPO, "examples", "build", "bench_host")
    if not os.path.exists(exe):
        return None
    n, ih, iw = wl.n, wl.images.shape[1], wl.images.shape[2]
    with tempfile.NamedTemporaryFile(suffix=".bgr", delete=False) as fh:
        np.ascontiguousarray(wl.images[:n]).tofile(fh)
        path = fh.name
    try:
        r = subprocess.run([exe, wl.model, path, str(n), str(iw), str(ih), str(reps)], capture_output=True, text=True,
                           timeout=300)
    finally:
        os.unlink(path)
    if r.returncode != 0:
        return {"error": r.stderr.strip()[-300:]}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    d["note"] = ("examples/bench_host.cpp: FaceForest::analyzeFaces (C++ shim -> ffd_analyze_faces) on pageable "
                 "host crops, median of %d batch calls; latency = analyzeFace per call, median of 50" % reps)
    return d


def evaluate_mt_path(wl):
    """The reference's low-level call pattern (getFacialFeaturesVotesMT, src/face_utils.cpp:244-302) from C++
    (examples/evaluate_mt.cpp through include/FaceForest.hpp): ImageSample on the device, one
    Forest<MPSample>::evaluateMT per patch (1,024 calls on copies of the forest), the vote filter, MeanShift per
    landmark, for face 0 of the workload; timings of the third repetition.  A child process, run before this one
    initialises the GPU."""
    import tempfile
    exe = os.path.join(REPO, "examples", "build", "evaluate_mt")
    if not os.path.exists(exe):
        return None
    img, box = wl.face(0)
    ih, iw = img.shape[:2]
    with tempfile.NamedTemporaryFile(suffix=".bgr", delete=False) as fh:
        np.ascontiguousarray(img).tofile(fh)
        path = fh.name
    try:
        r = subprocess.run([exe, wl.model, "--crop", path, str(iw), str(ih)] + [str(int(v)) for v in box],
                           capture_output=True, text=True, timeout=300)
    finally:
        os.unlink(path)
    if r.returncode != 0:
        return {"error": r.stderr.strip()[-300:]}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    keep = ("patches", "trees", "sample_ms", "first_call_ms", "other_calls_mean_us", "all_calls_ms", "vote_filter_ms",
            "meanshift_ms", "cold_first_call_ms", "reps")
    out = {k: d[k] for k in keep}
    out["per_call_us"] = round(d["all_calls_ms"] * 1e3 / d["patches"], 4)
    out["note"] = ("examples/evaluate_mt.cpp: Forest<MPSample>::evaluateMT once per patch as face_utils.cpp:267-274; "
                   "the first call of a sample evaluates its patch grid in one launch (ffd_sample_eval_grid), the "
                   "others read that result")
    return out


def single_face_latency(ff, wl, reps=50):
    """The reference's call pattern (eval_ffd.cpp:89): one analyzeFace per call, host image in,
    host record out, through ffd_analyze_faces (the C ABI the C++ shim calls)."""
    img, box = wl.face(0)
    ff.analyzeFace(img, box)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ff.analyzeFace(img, box)
        ts.append((time.perf_counter() - t0) * 1e3)
    return {"median_ms": round(float(np.median(ts)), 3), "min_ms": round(float(np.min(ts)), 3), "calls": reps}


def records_per_rank(n_local, world, dev):
    """Records each rank contributes to the gather: the largest local face count over the ranks
    (shards are padded to it), so no rank writes or gathers past its buffer when the counts differ
    (uneven frame shards, or --detect finding different numbers of faces per rank)."""
    if world == 1:
        return n_local
    import torch
    import torch.distributed as dist
    t = torch.tensor([n_local], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    per = int(t.item())
    assert n_local <= per
    return per


def launch_ranks(n):
    """Start n ranks of this script under torch.distributed.run as a child process (nothing in this
    process has touched the GPU) and return the child's exit status."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def dry_run(args, world, rank):
    """The N-rank path without a GPU: gloo process group, each rank's shard of synthetic records
    (headpose = global face index), one gather to rank 0 (distributed.gather_records).  --uneven:
    rank r holds ceil(N / world) + r - world // 2 faces (as --detect or a ragged frame split gives),
    gathered with the padded per-rank size records_per_rank() chooses, as the GPU path does."""
    import torch
    import torch.distributed as dist

    import face_alignment_cvpr_2012_amd as ffd
    from face_alignment_cvpr_2012_amd.distributed import gather_records, shard_bounds
    dist.init_process_group("gloo")
    total = args.faces or 61
    rec = ffd.FACE_RECORD_BYTES
    ranks = [None] * world
    dist.all_gather_object(ranks, (rank, os.getpid()))
    if args.uneven:
        counts = [max(0, -(-total // world) + r - world // 2) for r in range(world)]
        lo, n_local = sum(counts[:rank]), counts[rank]
        total = sum(counts)
        per = records_per_rank(n_local, world, torch.device("cpu"))
        recs = np.zeros((per, rec), np.uint8)
        recs[:n_local, :4] = np.arange(lo, lo + n_local, dtype=np.float32).view(np.uint8).reshape(-1, 4)
        parts = [torch.empty(per * rec, dtype=torch.uint8) for _ in range(world)] if rank == 0 else None
        dist.gather(torch.from_numpy(recs.reshape(-1)), gather_list=parts, dst=0)
        got = torch.cat([p[: c * rec] for p, c in zip(parts, counts)]) if rank == 0 else None
    else:
        lo, hi = shard_bounds(total, world, rank)
        recs = np.zeros((hi - lo, rec), np.uint8)
        recs[:, :4] = np.arange(lo, hi, dtype=np.float32).view(np.uint8).reshape(-1, 4)
        got = gather_records(torch.from_numpy(recs.reshape(-1)), total, dst=0)
    if rank == 0:
        faces = ffd.faces_from_records(got.numpy().tobytes())
        ok = [f.headpose for f in faces] == [float(i) for i in range(total)]
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": sorted(r for r, _ in ranks),
                          "pids": len({p for _, p in ranks}), "faces": total, "gather_ok": ok}), flush=True)
    dist.destroy_process_group()


def run_group(args):
    """--group: the single-process multi-device shape of the C ABI (include/ffd.h
    ffd_group_*): one engine per device, faces sharded in contiguous blocks, the records gathered to
    device 0 with ONE RCCL gather and copied to the host.  A step = ffd_group_analyze_faces over
    --gpus x 4096 C2 crops from pageable host memory (host-inclusive, like the reference's C++
    caller); weak scaling.  The driver's N-GPU runs use the one-rank-per-GPU shape instead."""
    import torch

    import face_alignment_cvpr_2012_amd as ffd
    if args.workload != "c2":
        raise SystemExit("--group runs the c2 workload")
    faces = args.faces or 4096
    wl = make_workload("c2", 0, 1, faces * args.gpus, args.frames)
    n = wl.n
    # the C ABI call itself is timed: image descriptors, boxes and the record array are built once
    # (as a C++ caller holding its cv::Mat headers would), records decoded after the timed loop
    keep, cim = ffd._image_array([wl.images[i] for i in range(len(wl.images))])
    rects = ffd._packed_rects([tuple(int(v) for v in b) for b in wl.boxes])
    out = (ffd._Face * n)()
    grp = ffd.FaceForestGroup(list(range(args.gpus)), ffd.FaceForestOptions(model_path=wl.model))
    L = ffd.lib()

    def call():
        st = L.ffd_group_analyze_faces(grp._h, cim, len(keep), rects.ctypes.data, None, n, out)
        if st != 0:
            raise SystemExit("ffd_group_analyze_faces: " + L.ffd_group_last_error(grp._h).decode(errors="replace"))
    try:
        for _ in range(args.warmup):
            call()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            call()
        elapsed = time.perf_counter() - t0
        torch.cuda.synchronize()
    finally:
        grp.close()
    ok = sum(1 for r in out if r.status == 0)
    print(json.dumps({
        "metric": "faces/sec (whole node) on pretrained FFD forest; mean landmark px error",
        "value": round(n * args.steps / elapsed, 1), "unit": "faces/s", "n_gpus": args.gpus, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8/u16/i32/f32",
        "data": "synthetic (face_alignment_cvpr_2012_amd/synthetic.py) from the 20 bundled LFW faces",
        "config": {"workload": wl.describe, "faces_per_gpu": faces,
                   "parallelism": f"group x{args.gpus}: one process, ffd_group_analyze_faces (ncclCommInitAll), "
                                  "host crops in, host records out (host-inclusive)"},
        "records_ok": ok}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=("c2", "c3", "c4", "c5"), default="c2",
                    help="BASELINE.json config: c2 (default, the metric's), c3 1080p frames, c4 deep synthetic "
                         "forest, c5 crowd")
    ap.add_argument("--faces", type=int, default=None, help="c2/c4: faces per GPU per step (4096 / 1024)")
    ap.add_argument("--frames", type=int, default=512, help="c3: frames per step (whole job)")
    ap.add_argument("--detect", action="store_true",
                    help="c3: boxes from the GPU Haar detector (FaceForest::detectFace) inside the timed step "
                         "instead of the known paste boxes")
    ap.add_argument("--chunk", type=int, default=0, help="faces per pipeline launch (0 = whole batch)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-paths", action="store_true", help="skip the host-inclusive and latency lines")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU-baseline work")
    ap.add_argument("--dry-run", action="store_true", help="launcher + gather only, gloo, no GPU")
    ap.add_argument("--group", action="store_true",
                    help="ONE process driving --gpus devices through the C ABI's ffd_group_analyze_faces "
                         "(ncclCommInitAll, host crops in / host records out) instead of one rank per GPU")
    ap.add_argument("--uneven", action="store_true", help="--dry-run: a different face count on every rank")
    args = ap.parse_args()

    if args.group:
        return run_group(args)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))  # one process per GPU, started before any GPU call
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (one rank per GPU)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)

    import torch
    import torch.distributed as dist

    import face_alignment_cvpr_2012_amd as ffd

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    faces = args.faces or (1024 if args.workload == "c4" else 4096)
    wl = make_workload(args.workload, rank, world, faces, args.frames)
    cxx_host = eval_mt = None
    if world == 1 and wl.name == "c2" and not args.no_host_paths:
        cxx_host = cxx_host_path(wl)  # child processes, before this one initialises the GPU
        eval_mt = evaluate_mt_path(wl)
    n = wl.n
    n_img, ih, iw = wl.n_images, wl.images.shape[1], wl.images.shape[2]
    d_images = torch.from_numpy(np.ascontiguousarray(wl.images)).to(dev)
    if n_img > len(wl.images):
        reps = -(-n_img // len(wl.images))
        d_images = d_images.repeat(reps, 1, 1, 1)[:n_img].contiguous()
    rec = ffd.FACE_RECORD_BYTES
    per = records_per_rank(n, world, dev)
    d_out = torch.zeros(max(1, per) * rec, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    chunk = args.chunk if 0 < args.chunk < n else 0  # 0: engine default (FFD_CHUNK)
    mp = ffd.MultiPartEstimatorOption(step_size=wl.mp_steps[0], step_size_y=wl.mp_steps[1])
    ff = ffd.FaceForest(ffd.FaceForestOptions(model_path=wl.model, device=local, max_chunk_faces=chunk, mp_option=mp))
    geo = [ff.geometry(int(b[2]), int(b[3])) for b in wl.boxes[:256]]
    mean_wh = (float(np.mean([g[0] for g in geo])), float(np.mean([g[1] for g in geo])))
    d_root = None
    rccl_ranks = None  # no communicator at N = 1 (nothing to gather)
    if world > 1:
        # the engines join one RCCL communicator inside libffd.so (ffd_engine_join); the 128-byte id
        # travels over the launcher's process group
        cid = torch.tensor(list(ffd.comm_id() if rank == 0 else bytes(ffd.COMM_ID_BYTES)), dtype=torch.uint8,
                           device=dev)
        dist.broadcast(cid, 0)
        ff.join(bytes(cid.cpu().tolist()), world, rank)
        rccl_ranks, rccl_rank = ff.comm_info()  # ncclCommCount / ncclCommUserRank on libffd.so's communicator
        if (rccl_ranks, rccl_rank) != (world, rank):
            raise SystemExit(f"bench.py: libffd.so's RCCL communicator has {rccl_ranks} ranks (this rank {rccl_rank}), "
                             f"expected {world} (rank {rank})")
        if rank == 0:
            d_root = torch.zeros(world * per * rec, dtype=torch.uint8, device=dev)

    if args.detect:
        if wl.name != "c3":
            raise SystemExit("--detect applies to the c3 (1080p frames) workload")
        # analyzeImage (FaceForest.cpp:161-181): the frames' faces are whatever the detector finds
        det_boxes, det_img = ff.detect_device(d_images.data_ptr(), iw * ih * 3, iw, ih, iw * 3, n_img)
        n_det = torch.tensor([len(det_boxes)], dtype=torch.int64, device=dev)
        if world > 1:
            dist.all_reduce(n_det)
        wl.total_faces = int(n_det.item())
        wl.boxes, wl.box_img = det_boxes, det_img
        wl.describe += "; boxes from the GPU Haar detector inside the step (detectFace on every frame)"
        n = wl.n
        per = records_per_rank(n, world, dev)
        d_out = torch.zeros(max(1, per) * rec, dtype=torch.uint8, device=dev)
        if world > 1 and rank == 0:
            d_root = torch.zeros(world * per * rec, dtype=torch.uint8, device=dev)

    def step():
        boxes, box_img = wl.boxes, wl.box_img
        if args.detect:
            boxes, box_img = ff.detect_device(d_images.data_ptr(), iw * ih * 3, iw, ih, iw * 3, n_img, cap=len(wl.boxes))
        ff.analyze_device(d_images.data_ptr(), iw * ih * 3, iw, ih, iw * 3, n_img, boxes, box_img,
                          d_out.data_ptr())
        if world > 1:  # ONE RCCL gather of the ffd_face records to rank 0 (faces sharded, no other exchange)
            ff.gather(d_out.data_ptr(), per, d_root.data_ptr() if d_root is not None else None, 0)
        ff.synchronize()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    px = landmark_error(wl, d_out) if rank == 0 else None

    ff.set_profiling(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    stages = ff.stage_times()
    ff.set_profiling(False)
    host_incl = latency = None
    if world == 1 and wl.name == "c2" and not args.no_host_paths:
        host_incl = host_inclusive(ff, wl, iw, ih, args.steps, args.warmup)
        latency = single_face_latency(ff, wl)
    detect_ms = None
    if args.detect:  # the detector alone, same frames (its share of the step)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            ff.detect_device(d_images.data_ptr(), iw * ih * 3, iw, ih, iw * 3, n_img, cap=len(wl.boxes))
        detect_ms = (time.perf_counter() - t1) / args.steps * 1e3
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if rank == 0:
        total_faces = wl.total_faces * args.steps
        value = total_faces / elapsed
        dom = max((k for k in stages if stages[k][1] > 0), key=lambda k: stages[k][0])
        ms_total, launches = stages[dom]
        avg_ms = ms_total / launches
        faces_per_launch = n * args.steps / launches  # one launch covers one chunk of faces
        W, H = mean_wh
        n_hp = float(np.mean([g[2] for g in geo])) if geo else 0.0
        n_mp = float(np.mean([g[3] for g in geo])) if geo else 0.0
        amount, unit, bound = stage_work(dom, faces_per_launch, W=W, H=H, n_hp=n_hp, n_mp=n_mp)
        achieved = amount / (avg_ms / 1e3)
        traffic = measured_traffic(dom, faces_per_launch) if wl.name == "c2" else None  # PMC bytes/launch
        traffic_raw = measured_traffic(dom, faces_per_launch, key="traffic_bytes_uncorrected") if wl.name == "c2" else None
        if traffic is not None:
            traffic = int(traffic)
        peak = FP32_PEAK_TFLOPS if unit == "TFLOP/s" else HBM_PEAK_GBS
        # B_face = S_in + 2*38*(W+1)*(H+1)*4 + S_out (C2: 4,893,904 B)
        s_in = iw * ih * 3 * n_img / max(1, n)
        b_face = int(round(s_in + 2 * 38 * (W + 1) * (H + 1) * 4 + 100))
        if wl.name == "c4":  # + forest gather P*T*(16 B * depth + 48 B)
            b_face += int(round(n_mp * 20 * (16 * 20 + 48)))
        out = {
            "metric": "faces/sec (whole node) on pretrained FFD forest; mean landmark px error",
            "value": round(value, 1),
            "unit": "faces/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": wl.scaling,
            "vs_baseline": None,
            "dtype": "u8/u16/i32/f32",
            "data": "synthetic (face_alignment_cvpr_2012_amd/synthetic.py) from the 20 bundled LFW faces; "
                    "pretrained reference forests converted to model/ffd_model.bin",
            "config": {"workload": wl.describe, "faces_per_gpu": n, "mean_face": [round(W, 1), round(H, 1)],
                       "parallelism": f"faces sharded x{world}"},
            "rccl_ranks": rccl_ranks,
            "landmark_px_error_vs_cpu": px["vs_cpu_px"],
            "landmark_px_error": px,
            "roofline": {"bound": bound, "kernel": dom, "achieved": round(achieved, 2), "peak": peak, "unit": unit,
                         "frac": round(achieved / peak, 4), "traffic": traffic,
                         "avg_launch_ms": round(avg_ms, 4), "faces_per_launch": faces_per_launch,
                         "algorithmic_bytes": int(amount * 1e9) if unit == "GB/s" else None,
                         "traffic_unit": "bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                         "traffic_uncorrected": int(traffic_raw) if traffic_raw else None,
                         "traffic_note": "FETCH_SIZE x2 is the guide's correction for wide streaming reads; this kernel "
                                         "also gathers 16-B node records, so its HBM bytes lie between "
                                         "traffic_uncorrected (FETCH_SIZE x1) and traffic"},
            "path_hbm_roofline": {"b_face": b_face, "achieved_GBs": round(value * b_face / 1e9, 1),
                                  "frac": round(value * b_face / 1e9 / HBM_PEAK_GBS, 4)},
            "stage_ms_per_step": {k: round(v[0] / max(1, args.steps), 3) for k, v in stages.items()},
        }
        if wl.name == "c2":  # the traversals' gather-path figure beside the HBM one (VERDICT r5 "next" #3)
            n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
            g = gather_figure(dom, avg_ms, faces_per_launch, n_cu)
            if g is not None:
                out["roofline"]["gather"] = g
            hs = stages.get("headpose_traverse")
            if hs and hs[1] > 0:
                gh = gather_figure("headpose_traverse", hs[0] / hs[1], n * args.steps / hs[1], n_cu)
                if gh is not None:
                    out["roofline"]["gather_headpose"] = gh
        # the Gabor stage's FP32 fraction beside the HBM figure, per scale
        gab = {}
        for k, (ms_k, nl) in stages.items():
            if k.startswith("gabor_") and ms_k > 0:
                w = int(k.split("_")[1].split("x")[0])
                fpp = gabor_flops_per_pixel(w, W)
                tf = n * args.steps * W * H * fpp / (ms_k / 1e3) / 1e12
                gab[k] = {"flops_per_px": round(fpp, 1), "tflops": round(tf, 2), "fp32_frac": round(tf / FP32_PEAK_TFLOPS, 4)}
        if gab:
            tot_ms = sum(stages[k][0] for k in gab) / max(1, args.steps)
            tot_tf = sum(n * W * H * gabor_flops_per_pixel(int(k.split("_")[1].split("x")[0]), W) for k in gab) / (tot_ms / 1e3) / 1e12
            out["gabor_fp32"] = {"per_scale": gab, "all_scales_ms": round(tot_ms, 3), "tflops": round(tot_tf, 2),
                                 "fp32_frac": round(tot_tf / FP32_PEAK_TFLOPS, 4), "peak_tflops": FP32_PEAK_TFLOPS}
        if wl.name == "c4":  # faces/s, patches/s, HBM fraction
            out["c4"] = {"patches_per_face": round(n_mp, 1), "patches_per_s": round(value * n_mp, 1),
                         "walks_per_s": round(value * n_mp * 20, 1), "forest_depth": 20}
        if host_incl is not None:
            # SURVEY.md §8(d)'s rule (H2D of the batch -> D2H of the records), same steps and warm-ups as `value`;
            # `value` is the device-resident throughput (inputs already in HBM, results left there)
            host_incl["rule"] = "SURVEY.md 8(d): H2D of the batch to D2H of results"
            out["host_inclusive"] = host_incl
            out["headline"] = ("value = device-resident throughput (batch in HBM); host_inclusive.value = the "
                               "SURVEY 8(d) H2D->D2H figure at the same steps / warm-ups")
            out["analyze_face_latency"] = latency
        if cxx_host is not None:
            out["cxx_host_path"] = cxx_host
            if host_incl is not None and "batch_faces_per_s" in cxx_host:
                cxx_host["vs_host_inclusive"] = round(cxx_host["batch_faces_per_s"] / host_incl["value"], 3)
        if eval_mt is not None:
            out["evaluate_mt_path"] = eval_mt
            if "all_calls_ms" in eval_mt:
                per_face_us = elapsed / total_faces * 1e6  # the batched path's per-face cost
                eval_mt["batched_per_face_us"] = round(per_face_us, 3)
                eval_mt["calls_vs_batched_per_face"] = round(eval_mt["all_calls_ms"] * 1e3 / per_face_us, 2)
        if detect_ms is not None:
            out["detect"] = {"frames_per_step": wl.n_images * world, "faces_found": wl.total_faces,
                             "detect_ms_per_step": round(detect_ms, 3),
                             "frames_per_s": round(wl.n_images * world / (detect_ms / 1e3), 1)}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(wl, args.cpu_budget)
        print(json.dumps(out), flush=True)
    ff.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
