"""Line locality of k_traverse's record gathers, simulated on the CPU (round 6).

For C2 faces (synthetic.make_crops, the bench's seed) the oracle supplies the 38 integral channels and the
selected FFD trees; every (patch, tree) walk is replayed on the model's pre-order node arrays
(Tree::evaluateMT, Tree.hpp:173-191; ImageSample::evalTest, ImageSample.cpp:48-63) and mapped to the kernel's
lanes exactly as k_traverse<FFD, 5, 5> deals them (walker thread = item = t * 25 + patch-in-block, waves of 64).
For each wave-level gather instruction of the deep loop (levels below the LDS tree tops) it counts the active
lanes and the distinct 128-byte lines their records fall in, under a record layout:

  dfs      the shipped depth-first pair layout (ffd_host::build_pair_records)
  <other>  candidate layouts (see LAYOUTS)

Usage: python tools/walk_locality.py [--faces N] [--layouts dfs,...] [--json out.json]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from face_alignment_cvpr_2012_amd import model as fmodel  # noqa: E402
from face_alignment_cvpr_2012_amd.synthetic import make_crops  # noqa: E402
import oracle  # noqa: E402

PATCH, TOPL = 31, 3  # patch, tree-top levels held in LDS (0..2)
KINDS = {"ffd": dict(prefix="mp", step=3, gx=5, gy=5, walkers=512),  # k_traverse<FFD, 5, 5>
         "hp": dict(prefix="hp", step=4, gx=5, gy=4, walkers=320)}   # k_traverse<HP, 5, 4>


def tree_structure(m, prefix):
    """Per tree: (b, e) node range; global arrays right child (pre-order), depth, internal rank."""
    off = m[prefix + ".tree_node_off"].astype(np.int64)
    leaf = m[prefix + ".node_leaf"]
    n = leaf.size
    right = np.full(n, -1, np.int64)
    depth = np.zeros(n, np.int32)
    rank = np.full(n, -1, np.int64)
    for t in range(off.size - 1):
        b, e = int(off[t]), int(off[t + 1])
        stack = []  # internal nodes waiting for their right child
        r = 0
        lf = leaf[b:e]
        for i in range(e - b):
            g = b + i
            if i > 0:
                # node i is the left child of i-1 if i-1 is internal, else the right child of the stack top
                if lf[i - 1] < 0:
                    depth[g] = depth[g - 1] + 1
                else:
                    p = stack.pop()
                    right[p] = g
                    depth[g] = depth[p] + 1
            if lf[i] < 0:
                stack.append(g)
                rank[g] = r
                r += 1
        assert not stack
    return off, right, depth, rank


def dfs_pair_index(m, prefix, off, rank):
    """Global pair index of each internal node's children pair in the shipped layout: tree base + 1 + rank."""
    leaf = m[prefix + ".node_leaf"]
    base = np.zeros(off.size - 1, np.int64)
    acc = 0
    for t in range(off.size - 1):
        base[t] = acc
        acc += 1 + int((leaf[int(off[t]):int(off[t + 1])] < 0).sum())
    tree_of = np.repeat(np.arange(off.size - 1), np.diff(off))
    return base[tree_of] + 1 + rank, acc


def face_walks(m, prefix, right, ch, trees, nx, ny, step):
    """Node sequence of every walk: paths[t][patch] -> array of node ids (pre-order, global)."""
    STEP = step
    sp = m[prefix + ".node_split"].astype(np.int64)
    leaf = m[prefix + ".node_leaf"]
    off = m[prefix + ".tree_node_off"]
    P = nx * ny
    xs = (np.arange(P) // ny) * STEP  # patch i = xi * ny + yi (reference order)
    ys = (np.arange(P) % ny) * STEP
    out = []
    for t in trees:
        cur = np.full(P, int(off[t]), np.int64)
        path = [cur.copy()]
        alive = leaf[cur] < 0
        while alive.any():
            s = sp[cur]
            c = s[:, 0]

            cl = np.where(alive, c, 0)
            s = np.where(alive[:, None], s, np.array([[0, 0, 0, 1, 1, 0, 0, 1, 1, 0]]))
            c = cl
            p1 = _mean(ch, c, xs + s[:, 1], ys + s[:, 2], s[:, 3], s[:, 4])
            p2 = _mean(ch, c, xs + s[:, 5], ys + s[:, 6], s[:, 7], s[:, 8])
            go_left = (p1 - p2) <= s[:, 9]
            nxt = np.where(go_left, cur + 1, right[cur])
            cur = np.where(alive, nxt, cur)
            path.append(np.where(alive, cur, -1))
            alive = alive & (leaf[np.maximum(cur, 0)] < 0)
        out.append(np.stack(path, 1))  # [P][steps], -1 after the leaf
    return out


def _mean(ch, c, x, y, w, h):
    a = ch[c, y, x].astype(np.int64)
    b = ch[c, y, x + w].astype(np.int64)
    cc = ch[c, y + h, x].astype(np.int64)
    d = ch[c, y + h, x + w].astype(np.int64)
    return (d - b - cc + a) // (w * h)


def treelet_lines(m, prefix, off, right, depth, levels=3, top=TOPL):
    """Line of each internal node's children pair when every `levels` pair levels below the LDS tops form one
    heap-ordered treelet per 128-byte line (slot 0 its root's pair, then 2, 4, ...): line id per node, lines used."""
    leaf = m[prefix + ".node_leaf"]
    n = leaf.size
    line = np.full(n, -1, np.int64)
    nl = 0
    for t in range(off.size - 1):
        b, e = int(off[t]), int(off[t + 1])
        d = depth[b:e]
        lf = leaf[b:e] < 0
        for i in range(e - b):
            if not lf[i] or d[i] < top:
                continue
            if (d[i] - top) % levels == 0:
                line[b + i] = nl
                nl += 1
        # propagate: a node below a treelet root inherits its ancestor's line (pre-order: parent before child)
        stack = []
        for i in range(e - b):
            g = b + i
            while stack and stack[-1][1] <= 0:
                stack.pop()
            if stack:
                par = stack[-1][0]
                stack[-1][1] -= 1
            else:
                par = -1
            if lf[i]:
                if d[i] >= top and line[g] < 0 and par >= 0:
                    line[g] = line[par]
                stack.append([g, 2])
    return line, nl


def simulate(paths, nx, ny, pair_line, depth, T, gx, gy, walkers, waves_lanes=64, l1_lines=256):
    """Per wave instruction of the deep loop: (depth band, active lanes, distinct lines, L1 misses).  L1: an LRU of
    l1_lines 128-B lines per CU shared by the block's walker waves, which issue their k-th gathers in turn."""
    from collections import OrderedDict
    recs = []
    gbx, gby = (nx + gx - 1) // gx, (ny + gy - 1) // gy
    GG = gx * gy
    for by in range(gby):
        for bx in range(gbx):
            items = GG * T
            wl = []
            l1 = OrderedDict()
            for w0 in range(0, walkers, waves_lanes):
                lanes = []
                for item in range(w0, min(w0 + waves_lanes, items)):
                    t, pl = item // GG, item % GG
                    xi, yi = bx * gx + pl % gx, by * gy + pl // gx
                    if xi >= nx or yi >= ny:
                        continue
                    seq = paths[t][xi * ny + yi]
                    seq = seq[seq >= 0]
                    # gathers: the children pair of every internal node at depth >= TOPL on the path
                    inner = seq[:-1]
                    g = inner[depth[inner] >= TOPL]
                    lanes.append(pair_line(g))
                if lanes:
                    wl.append(lanes)
            k = 0
            while True:
                any_ = False
                for lanes in wl:
                    act = [ln[k] for ln in lanes if len(ln) > k]
                    if not act:
                        continue
                    any_ = True
                    u = set(act)
                    miss = 0
                    for x in u:
                        if x in l1:
                            l1.move_to_end(x)
                        else:
                            miss += 1
                            l1[x] = 1
                            if len(l1) > l1_lines:
                                l1.popitem(last=False)
                    recs.append((TOPL + k, len(act), len(u), miss))
                if not any_:
                    break
                k += 1
    return recs


def summarise(recs):
    a = np.array(recs, np.int64)
    out = {"instr": int(len(a)), "lane_gathers": int(a[:, 1].sum()), "lines": int(a[:, 2].sum()),
           "l1_misses": int(a[:, 3].sum())}
    out["lanes_per_instr"] = out["lane_gathers"] / out["instr"]
    out["lines_per_instr"] = out["lines"] / out["instr"]
    out["l1_miss_lines_per_instr"] = out["l1_misses"] / out["instr"]
    bands = {}
    for lo, hi in ((3, 6), (6, 9), (9, 12), (12, 15), (15, 21)):
        sel = (a[:, 0] >= lo) & (a[:, 0] < hi)
        if sel.any():
            bands[f"{lo}-{hi - 1}"] = {"instr": int(sel.sum()), "lanes_per_instr": float(a[sel, 1].mean()),
                                       "lines_per_instr": float(a[sel, 2].mean()),
                                       "l1_miss_lines_per_instr": float(a[sel, 3].mean())}
    out["by_depth"] = bands
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--faces", type=int, default=8)
    ap.add_argument("--kind", choices=("ffd", "hp", "both"), default="both")
    ap.add_argument("--layouts", default="dfs,treelet3,treelet2")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    m = fmodel.load(os.path.join(REPO, "model", "ffd_model.bin"))
    oracle.load_model(os.path.join(REPO, "model", "ffd_model.bin"))
    crops, _ = make_crops(args.faces, seed=2012)
    traces = [oracle.analyze_face(crops[f], (0, 0, 150, 150), trace=True) for f in range(args.faces)]
    res = {"faces": args.faces, "source": "tools/walk_locality.py: C2 crops (synthetic.make_crops seed 2012), oracle "
           "channels and tree selection, k_traverse's lane mapping; lines = distinct 128-B lines per wave-level gather "
           "instruction; l1 = misses of an LRU of 256 lines per CU shared by the walker waves (staging not modelled)"}
    for kind in (("ffd", "hp") if args.kind == "both" else (args.kind,)):
        K = KINDS[kind]
        off, right, depth, rank = tree_structure(m, K["prefix"])
        pidx, npairs = dfs_pair_index(m, K["prefix"], off, rank)
        layouts = {"dfs": lambda g: list(pidx[g] * 16 // 128)}
        foot = {"dfs": npairs * 16}
        for name, lv in (("treelet3", 3), ("treelet2", 2)):
            if name in args.layouts.split(","):
                tl, nl = treelet_lines(m, K["prefix"], off, right, depth, lv)
                layouts[name] = (lambda tl_: (lambda g: list(tl_[g])))(tl)
                foot[name] = nl * 128
        allrec = {k: [] for k in layouts}
        walks = 0
        for face, tr in traces:
            ch = tr["channels"]
            W, H = face["face_w"], face["face_h"]
            nx = len(range(0, W - PATCH, K["step"]))
            ny = len(range(0, H - PATCH, K["step"]))
            trees = [int(t) for t in tr["trees"]] if kind == "ffd" else list(range(off.size - 1))
            paths = face_walks(m, K["prefix"], right, ch, trees, nx, ny, K["step"])
            if kind == "ffd":  # the walks end at the oracle's leaves
                leaf = m["mp.node_leaf"]
                got = np.stack([leaf[p[np.arange(p.shape[0]), (p >= 0).sum(1) - 1]] for p in paths], 1)
                assert np.array_equal(got, tr["mp_leaves"]), "walk replay differs from the oracle"
            walks += nx * ny * len(trees)
            for k, fn in layouts.items():
                allrec[k] += simulate(paths, nx, ny, fn, depth, len(trees), K["gx"], K["gy"], K["walkers"])
        out = {k: summarise(v) for k, v in allrec.items()}
        for k in out:
            out[k]["footprint_bytes"] = int(foot[k])
            out[k]["lane_gathers_per_face"] = out[k]["lane_gathers"] / args.faces
            out[k]["instr_per_face"] = out[k]["instr"] / args.faces
        out["walks_per_face"] = walks / args.faces
        res[kind] = out
    print(json.dumps(res, indent=1))
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
