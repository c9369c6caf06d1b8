"""Generate tests/golden/train_hp_golden.npz: a head-pose tree grown by the CPU restatement
(oracle/ffd_train_oracle.cpp, Tree<HeadPoseSample>) at the reference's config_headpose.txt shape
(max_depth 15, min_patches 20, 25 thresholds, 31-pixel patches of a 125-pixel face, 20 % background
patches) with fewer stripes, patches and images, from synthetic.headpose_training_images.  Parity with
the reference is unpinned (no LFW, no OpenCV/Boost, time(NULL) seeds): the golden pins the restatement,
and the GPU trainer is checked against it (tests/test_training_hp.py).

    python tests/golden/make_train_hp_golden.py
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle  # noqa: E402
from face_alignment_cvpr_2012_amd.synthetic import headpose_training_images  # noqa: E402

N_IMAGES = 20
PARAM = dict(max_depth=15, min_patches=20, ntests=200, npatches=100, tree_seed=3, split_seed=1346000000)

if __name__ == "__main__":
    images, faces, poses = headpose_training_images(N_IMAGES)
    t = time.time()
    a = oracle.train_hp_tree(images, faces, poses, **PARAM)
    print(f"oracle: {time.time() - t:.1f} s, {len(a['node_leaf'])} nodes, {len(a['leaf_n'])} leaves, "
          f"i_node {a['i_node']}, {len(a['samples'])} patches")
    np.savez_compressed(os.path.join(HERE, "train_hp_golden.npz"), n_images=np.int32(N_IMAGES),
                        param=np.array([PARAM[k] for k in ("max_depth", "min_patches", "ntests", "npatches",
                                                           "tree_seed", "split_seed")], np.int64),
                        i_node=np.int64(a["i_node"]),
                        **{k: a[k] for k in ("node_leaf", "node_split", "node_info", "node_mode", "leaf_n", "leaf_fg",
                                             "leaf_labels", "samples")})
