"""Offline study (CPU, oracle channels): how often a split rectangle's sum needs its 17th bit.

The traversal reads each rectangle of a node test from u16 integrals (mod 2^16).  A rectangle of
area A <= 257 has R = sum <= 255 A < 2^16, so its 4-corner sum mod 2^16 is exact; larger ones need the
middle integral row today (6 reads instead of 4).  This tool walks the FFD trees of C2 faces exactly
as Tree::evaluateMT does (oracle channels, model arrays) and, per visit, classifies each rectangle:
  small      A <= 257
  bound      A > 257 but R_mod + 65536 > A * max(channel pixel values in the block window): the
             high candidate is impossible, so 4 reads are exact
  decided    both candidates (R_mod, R_mod + 65536) give the same test outcome
  ambiguous  neither: the middle row is needed
and reports the fraction of wave-steps (64 consecutive walks of a 5x5 block, one visit each) in
which some lane is ambiguous.

usage: python tools/sim_rect_bits.py [--faces 8]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def children(split, leaf, off):
    """left/right child indices of pre-order node records."""
    n = len(leaf)
    left = np.full(n, -1, np.int64)
    right = np.full(n, -1, np.int64)
    for t in range(len(off) - 1):
        b, e = int(off[t]), int(off[t + 1])
        stack = []  # nodes waiting for their right child
        for i in range(b, e):
            if stack:
                p = stack[-1]
                if left[p] == -1:
                    left[p] = i
                else:
                    right[p] = i
                    stack.pop()
            if leaf[i] < 0:
                stack.append(i)
    return left, right


MODE = "exact"


def main():
    global MODE
    ap = argparse.ArgumentParser()
    ap.add_argument("--faces", type=int, default=8)
    ap.add_argument("--mode", default="exact", choices=("exact", "mask"))
    args = ap.parse_args()
    MODE = args.mode
    import oracle
    from face_alignment_cvpr_2012_amd import model as fm
    from face_alignment_cvpr_2012_amd.synthetic import make_crops

    path = os.path.join(REPO, "model", "ffd_model.bin")
    m = fm.load(path)
    oracle.load_model(path)
    split = m["mp.node_split"].astype(np.int64)
    leaf = m["mp.node_leaf"]
    off = m["mp.tree_node_off"]
    left, right = children(split, leaf, off)
    crops, _ = make_crops(args.faces, seed=2012)
    tot = {"visits": 0, "rects": 0, "small": 0, "bound": 0, "decided": 0, "ambiguous": 0}
    wave_steps = wave_amb = wave_amb_nobound = 0
    for k in range(args.faces):
        face, tr = oracle.analyze_face(crops[k], (0, 0, 150, 150), trace=True)
        ch = tr["channels"].astype(np.int64)  # [38][H+1][W+1] exact integrals
        H, W = ch.shape[1] - 1, ch.shape[2] - 1
        trees = tr["trees"]
        roots = off[trees]
        nx = ny = 32
        # pixel values per channel (second differences of the integral)
        pix = ch[:, 1:, 1:] - ch[:, :-1, 1:] - ch[:, 1:, :-1] + ch[:, :-1, :-1]
        for bx in range(0, nx, 5):
            for by in range(0, ny, 5):
                px0, py0 = bx * 3, by * 3
                wmax = pix[:, py0:py0 + 44, px0:px0 + 44].reshape(38, -1).max(axis=1)
                # walks of the block in k_traverse's lane order: item = t * 25 + (dy * 5 + dx)
                items = [(t, bx + p % 5, by + p // 5) for t in range(len(trees)) for p in range(25)
                         if bx + p % 5 < nx and by + p // 5 < ny]
                node = np.array([roots[t] for t, _, _ in items])
                xs = np.array([x * 3 for _, x, _ in items])
                ys = np.array([y * 3 for _, _, y in items])
                alive = leaf[node] < 0
                while alive.any():
                    idx = np.nonzero(alive)[0]
                    nd = node[idx]
                    s = split[nd]
                    c = s[:, 0]
                    res = []
                    amb_lane = np.zeros(len(idx), bool)
                    amb_lane_nb = np.zeros(len(idx), bool)
                    cand = []
                    for r in range(2):
                        rx, ry, rw, rh = s[:, 1 + 4 * r], s[:, 2 + 4 * r], s[:, 3 + 4 * r], s[:, 4 + 4 * r]
                        x0, y0 = xs[idx] + rx, ys[idx] + ry
                        R = ch[c, y0 + rh, x0 + rw] - ch[c, y0, x0 + rw] - ch[c, y0 + rh, x0] + ch[c, y0, x0]
                        A = rw * rh
                        small = A <= 257
                        rmod = R & 0xFFFF
                        hi_possible = (rmod + 65536) <= 255 * A
                        bound_ok = (rmod + 65536) > A * wmax[c]
                        if MODE == "mask":  # window flag: channel max <= 135 (then every A <= 484 is bounded)
                            bound_ok = wmax[c] <= 135
                        cand.append((R // A, np.where(hi_possible, (rmod + 65536) // A, R // A), small, bound_ok,
                                     hi_possible))
                        tot["rects"] += len(idx)
                        tot["small"] += int(small.sum())
                        tot["bound"] += int((~small & (~hi_possible | bound_ok)).sum())
                    thr = s[:, 9]
                    (p1, p1h, s1, b1, h1), (p2, p2h, s2, b2, h2) = cand
                    # candidates for p1 - p2 (low/high of each when ambiguous)
                    need1 = ~s1 & h1 & ~b1
                    need2 = ~s2 & h2 & ~b2
                    lo1 = np.where(need1, np.minimum(p1, p1h), p1)
                    hi1 = np.where(need1, np.maximum(p1, p1h), p1)
                    lo2 = np.where(need2, np.minimum(p2, p2h), p2)
                    hi2 = np.where(need2, np.maximum(p2, p2h), p2)
                    dmin, dmax = lo1 - hi2, hi1 - lo2
                    decided = (dmax <= thr) | (dmin > thr)
                    if MODE == "mask":
                        decided = np.zeros_like(decided)
                    amb = (need1 | need2) & ~decided
                    tot["decided"] += int(((need1 | need2) & decided).sum())
                    tot["ambiguous"] += int(amb.sum())
                    nb1 = ~s1 & h1
                    nb2 = ~s2 & h2
                    # wave grouping: 64 consecutive items
                    for w0 in range(0, len(items), 64):
                        sel = (idx >= w0) & (idx < w0 + 64)
                        if sel.any():
                            wave_steps += 1
                            wave_amb += int(amb[sel].any())
                            wave_amb_nobound += int((nb1 | nb2)[sel].any())
                    tot["visits"] += len(idx)
                    go_left = (p1 - p2) <= thr
                    node[idx] = np.where(go_left, left[nd], right[nd])
                    alive = leaf[node] < 0
        print(f"face {k}: visits so far {tot['visits']}", flush=True)
    r = tot["rects"]
    print({k: (v / r if k in ("small", "bound", "decided", "ambiguous") else v) for k, v in tot.items()})
    print(f"ambiguous visits {tot['ambiguous'] / tot['visits']:.4f}; wave-steps with an ambiguous lane "
          f"{wave_amb / wave_steps:.4f}; with a big rectangle that has a possible high candidate "
          f"{wave_amb_nobound / wave_steps:.4f}")


if __name__ == "__main__":
    main()
