"""Walk statistics of the two traversals (k_traverse built with -DFFD_TRAV_STATS=1).

usage (GPU): FFD_LIBRARY=build/stats/libffd.so python tools/trav_stats.py [--faces 4096] [--out f.json]

Per traversal (head pose, FFD) it reports, from the kernel's per-(workgroup, block, wave) records:
  * walk length per block: mean over the block's walks vs the longest walk of the block;
  * visits split into LDS tree-top visits and deep visits (one pair-record fetch each);
  * cycles per block (period between a workgroup's consecutive windows), the walker waves' busy cycles,
    the stager's commit wait;
  * cycles per wave-step (a walker wave's walk cycles / its longest walk), lane activity
    (visits / (64 x longest walk per wave)), and cycles per visit per walker lane
    (walker lanes x block periods / visits).
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

ITERS, SLOTS = 1024, 9


def summarise_timing(rec, nw_waves):
    """FFD_TRAV_STATS=2 builds: per wave, cycles of the node tests and of the record waits over its deep
    steps (fields 2, 3), deep steps of its longest walk (field 6)."""
    wk = rec[:, :, :nw_waves, :].astype(np.float64)
    ok = wk[..., 5] > 0
    steps = wk[..., 6][ok].sum()
    return {"test_cycles_per_deep_step": float(wk[..., 2][ok].sum() / steps),
            "fetch_wait_cycles_per_deep_step": float(wk[..., 3][ok].sum() / steps),
            "walk_cycles_per_wave_mean": float(wk[..., 1][ok].mean())}


def summarise_phases(rec, nw_waves):
    """FFD_TRAV_STATS=3 builds: per wave, cycles of its walk phases (fields 2, 3, 4, 6) and the whole walk (1)."""
    wk = rec[:, :, :nw_waves, :].astype(np.float64)
    ok = wk[..., 5] > 0
    return {"walk": float(wk[..., 1][ok].mean()), "setup": float(wk[..., 2][ok].mean()),
            "top_levels": float(wk[..., 3][ok].mean()), "deep_levels": float(wk[..., 4][ok].mean()),
            "store": float(wk[..., 6][ok].mean())}


def summarise(rec, nw_waves, walker_lanes, per_lane=1):
    # rec: [wg][iter][slot][8] u32
    wk = rec[:, :, :nw_waves, :].astype(np.float64)
    st = rec[:, :, 8, :].astype(np.float64)
    walks = wk[..., 5]
    used = walks.sum(axis=2) > 0  # (wg, iter) blocks that walked
    t0 = rec[:, :, 0, 0].astype(np.int64)
    out = {}
    vis_top = wk[..., 2].sum(axis=2)[used]
    vis_deep = wk[..., 3].sum(axis=2)[used]
    nwalk = walks.sum(axis=2)[used]
    maxlen = wk[..., 4].max(axis=2)[used]
    mean_len = (vis_top + vis_deep) / np.maximum(nwalk, 1)
    out["blocks"] = int(used.sum())
    out["walks_per_block_mean"] = float(nwalk.mean())
    out["walk_len_mean"] = float(mean_len.mean())
    out["walk_len_block_max_mean"] = float(maxlen.mean())
    out["mean_over_max"] = float((mean_len / np.maximum(maxlen, 1)).mean())
    out["top_visits_per_walk"] = float(vis_top.sum() / nwalk.sum())
    out["deep_visits_per_walk"] = float(vis_deep.sum() / nwalk.sum())
    # block period: difference of consecutive t0 of one workgroup's walker wave 0 (32-bit clock)
    per = []
    busy = []
    steps = []
    act = []
    for g in range(rec.shape[0]):
        n = int(used[g].sum())
        if n < 3:
            continue
        t = t0[g, :n]
        d = (np.diff(t) & 0xFFFFFFFF).astype(np.float64)
        per.extend(d.tolist())
        for i in range(n):
            for w in range(nw_waves):
                if rec[g, i, w, 5] == 0:
                    continue
                busy.append(float(rec[g, i, w, 1]))
                ml = float(rec[g, i, w, 4])
                steps.append(float(rec[g, i, w, 1]) / max(ml, 1))
                act.append(float(rec[g, i, w, 2] + rec[g, i, w, 3]) / (64.0 * per_lane * max(ml, 1)))
    per = np.array(per)
    out["block_period_cycles_median"] = float(np.median(per))
    out["block_period_cycles_mean"] = float(per.mean())
    out["walker_wave_busy_cycles_mean"] = float(np.mean(busy))
    out["cycles_per_wave_step_mean"] = float(np.mean(steps))
    out["lane_activity_mean"] = float(np.mean(act))
    out["stager_commit_cycles_mean"] = float(st[..., 1][used].mean())
    out["cycles_per_visit_per_walker_lane"] = float(walker_lanes * per_lane * per.mean() / ((vis_top + vis_deep).mean()))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--faces", type=int, default=4096)
    ap.add_argument("--out", default="")
    ap.add_argument("--timing", action="store_true", help="FFD_TRAV_STATS=2 build: test / fetch-wait split")
    ap.add_argument("--phases", action="store_true", help="FFD_TRAV_STATS=3 build: walk phases")
    ap.add_argument("--dual", action="store_true", help="FFD_TRAV_DUAL build: 192 / 256 walker lanes, 2 walks each")
    ap.add_argument("--same-face", action="store_true", help="every face of the batch the same crop (L2-resident trees)")
    args = ap.parse_args()
    import torch

    import face_alignment_cvpr_2012_amd as ffd
    from face_alignment_cvpr_2012_amd.synthetic import make_crops

    L = ffd.lib()
    L.ffd_trav_stats_enable.restype = ctypes.c_int
    L.ffd_trav_stats_read.restype = ctypes.c_int
    L.ffd_trav_stats_read.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
    crops, _ = make_crops(1 if args.same_face else args.faces, seed=2012)
    if args.same_face:
        crops = np.repeat(crops, args.faces, axis=0)
    dev = torch.device("cuda:0")
    d_img = torch.from_numpy(np.ascontiguousarray(crops)).to(dev)
    rec = ffd.FACE_RECORD_BYTES
    d_out = torch.zeros(args.faces * rec, dtype=torch.uint8, device=dev)
    ff = ffd.FaceForest(ffd.FaceForestOptions(device=0))
    assert L.ffd_trav_stats_enable() == 0
    boxes = [(0, 0, 150, 150)] * args.faces
    box_img = np.arange(args.faces, dtype=np.int32)
    for _ in range(2):
        ff.analyze_device(d_img.data_ptr(), 150 * 150 * 3, 150, 150, 450, args.faces, boxes, box_img, d_out.data_ptr())
        ff.synchronize()
    ff.set_profiling(True)
    ff.analyze_device(d_img.data_ptr(), 150 * 150 * 3, 150, 150, 450, args.faces, boxes, box_img, d_out.data_ptr())
    ff.synchronize()
    stages = ff.stage_times()
    res = {"faces": args.faces, "library": ffd.library_path(), "stage_ms": stages}
    walkers = ((1, "headpose", 192), (0, "ffd", 256)) if args.dual else ((1, "headpose", 320), (0, "ffd", 512))
    pl = 2 if args.dual else 1
    for hp, name, nw in walkers:
        buf = np.zeros((256, ITERS, SLOTS, 8), dtype=np.uint32)
        assert L.ffd_trav_stats_read(hp, buf.ctypes.data, buf.nbytes) == 0
        res[name] = (summarise_timing(buf, nw // 64) if args.timing else
                     summarise_phases(buf, nw // 64) if args.phases else summarise(buf, nw // 64, nw, pl))
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
