"""Training throughput: one facial-feature tree at the reference's config_ffd.txt
(max_depth 20, min_patches 20, ntests 2500, 150 patches per image, 25 thresholds) on the GPU, and the CPU
restatement on a bounded sample of the same work, one JSON line.

Unit: stripe-sample evaluations per second = sum over the split-searched nodes of ntests x (node's
samples), each of which is one evalTest + its share of the sort and of the 25 thresholds' sequential
entropy sums (SplitGen.hpp:74-101,170-231).  The reference spends its training time there.

    python tools/train_bench.py [--images 200] [--cpu-images 6]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from face_alignment_cvpr_2012_amd.synthetic import training_rois  # noqa: E402


def searched_units(node_leaf, leaf_n, ntests, n_samples, min_patches, max_depth):
    """sum over split-searched nodes of ntests * n_node, from the pre-order arrays."""
    units, i, leaf_i = 0, 0, 0

    def walk(i, depth):
        nonlocal units
        if node_leaf[i] >= 0:
            n = int(leaf_n[node_leaf[i]])
            if n >= min_patches and depth < max_depth:  # searched, no valid split
                units += ntests * n
            return i + 1, n
        j, a = walk(i + 1, depth + 1)
        k, b = walk(j, depth + 1)
        units += ntests * (a + b)
        return k, a + b
    walk(0, 0)
    return units


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=200)
    ap.add_argument("--ntests", type=int, default=2500)
    ap.add_argument("--npatches", type=int, default=150)
    ap.add_argument("--cpu-images", type=int, default=6)
    ap.add_argument("--cpu-ntests", type=int, default=100)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    from face_alignment_cvpr_2012_amd.training import ForestParam, train_mp_tree
    rois, parts = training_rois(args.images)
    p = ForestParam(ntests=args.ntests, npatches=args.npatches)
    train_mp_tree(rois[:4], parts[:4], ForestParam(ntests=8, npatches=8, max_depth=4))  # warm-up (module load)
    t0 = time.perf_counter()
    t = train_mp_tree(rois, parts, p, tree_seed=1, split_seed=1346000000)
    wall = time.perf_counter() - t0
    a = t.arrays()
    units = searched_units(a["node_leaf"], a["leaf_n"], p.ntests, args.images * p.npatches, p.min_patches, p.max_depth)
    st = t.stats
    out = {"metric": "facial-feature tree training (one tree, config_ffd.txt)", "unit": "stripe-sample evals/s",
           "value": round(units / wall, 1), "tree_s": round(wall, 3), "images": args.images,
           "samples": args.images * p.npatches, "ntests": p.ntests, "nodes": t.num_nodes, "leaves": t.num_leaves,
           "levels": st["levels"], "items": st["items"], "stripe_sample_units": units,
           "phase_ms": {k: round(st[k], 1) for k in ("channels_ms", "search_ms", "partition_ms", "leaves_ms")}}
    if not args.no_cpu:
        import oracle
        cr, cp = rois[:args.cpu_images], parts[:args.cpu_images]
        t0 = time.perf_counter()
        b = oracle.train_mp_tree(cr, cp, ntests=args.cpu_ntests, npatches=p.npatches, tree_seed=1, split_seed=1346000000)
        cw = time.perf_counter() - t0
        cu = searched_units(b["node_leaf"], b["leaf_n"], args.cpu_ntests, len(cr) * p.npatches, 20, 20)
        out["cpu_baseline"] = {"value": round(cu / cw, 1), "unit": "stripe-sample evals/s", "cores": 1, "kind": "port",
                               "sample": f"oracle/ffd_train_oracle.cpp, one tree over {len(cr)} ROIs x {p.npatches} "
                                         f"patches, ntests {args.cpu_ntests}, {cw:.1f} s (incl. channels)"}
        out["vs_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
