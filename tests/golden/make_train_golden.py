"""Generate tests/golden/train_golden.npz: a facial-feature tree grown by the CPU restatement
(oracle/ffd_train_oracle.cpp) at the reference's config_ffd.txt shape (max_depth 20, min_patches 20,
25 thresholds, 31-pixel patches of a 125-pixel face) with fewer stripes and images, from
synthetic.training_rois.  Parity with the reference is unpinned (no LFW, no OpenCV/Boost, time(NULL)
seeds): the golden pins the restatement, and the GPU trainer is checked against it (tests/test_training.py).

    python tests/golden/make_train_golden.py
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle  # noqa: E402
from face_alignment_cvpr_2012_amd.synthetic import training_rois  # noqa: E402

N_IMAGES = 30
PARAM = dict(max_depth=20, min_patches=20, ntests=120, npatches=100, tree_seed=1, split_seed=1346000000)

if __name__ == "__main__":
    rois, parts = training_rois(N_IMAGES)
    t = time.time()
    a = oracle.train_mp_tree(rois, parts, **PARAM)
    print(f"oracle: {time.time() - t:.1f} s, {len(a['node_leaf'])} nodes, {len(a['leaf_n'])} leaves, i_node {a['i_node']}")
    np.savez_compressed(os.path.join(HERE, "train_golden.npz"), n_images=np.int32(N_IMAGES),
                        param=np.array([PARAM[k] for k in ("max_depth", "min_patches", "ntests", "npatches",
                                                           "tree_seed", "split_seed")], np.int64),
                        **{k: a[k] for k in ("node_leaf", "node_split", "node_info", "leaf_n", "leaf_fg", "leaf_offset",
                                             "leaf_var", "leaf_pf", "samples")})
