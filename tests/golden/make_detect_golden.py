"""Golden vectors for the Haar detector restatement: the oracle's detectFace
boxes (and raw candidate counts) on the 20 bundled fixture images and on 2 synthetic 1080p frames
(synthetic.make_frames(2)).  The restatement's parity with OpenCV is unpinned (no OpenCV in this
image); these pin the restatement itself against regressions, and the GPU tests compare the HIP
detector with the oracle directly.

    python tests/golden/make_detect_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import oracle  # noqa: E402
from face_alignment_cvpr_2012_amd import synthetic  # noqa: E402


def main():
    oracle.load_model(os.path.join(REPO, "model", "ffd_model.bin"))
    fx = synthetic.load_fixtures()
    out = {"fixtures": [], "frames": []}
    for img in fx["images"]:
        boxes, raw = oracle.detect_faces(img, raw=True)
        out["fixtures"].append({"boxes": boxes.tolist(), "n_raw": int(len(raw))})
    frames, _, _ = synthetic.make_frames(2)
    for fr in frames:
        boxes, raw = oracle.detect_faces(fr, raw=True)
        out["frames"].append({"boxes": boxes.tolist(), "n_raw": int(len(raw)), "raw_head": raw[:16].tolist()})
    json.dump(out, open(os.path.join(HERE, "detect_golden.json"), "w"))
    print("fixtures", len(out["fixtures"]), "frames", len(out["frames"]))


if __name__ == "__main__":
    main()
