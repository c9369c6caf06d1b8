"""Generate tests/golden/reference_pins.json: lines of the reference's OWN end-to-end output that
the restatement reproduces byte for byte (run in the build container only; the JSON is committed).

Source (reference, read-only): output/errors.txt, written by evalForest
(/root/reference/src/eval_ffd.cpp:102-121): one LFW test face per line, the 10 per-landmark
IOD-normalised errors of FaceForest::analyzeFace, C++ `ostream << float` format.

Method: for each of the 20 annotated faces the reference bundles (tests/golden/faces.npz,
data/imgs/index_random_subset.txt), run the CPU restatement (oracle/) with the annotated box,
format its errors exactly as eval_ffd does (face_alignment_cvpr_2012_amd/eval.py) and look the
line up in errors.txt.  Only faces of the reference's LFW test split appear there; every exact
match is recorded together with the best entry-wise overlap of the faces that do not match (so a
reader can see the other fixtures are absent from the test split, not near misses).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("FFD_REFERENCE", "/root/reference")
OUT = os.path.join(HERE, "reference_pins.json")


def main():
    sys.path.insert(0, REPO)
    import oracle
    from face_alignment_cvpr_2012_amd import eval as fe
    from face_alignment_cvpr_2012_amd.synthetic import load_fixtures

    oracle.load_model(os.path.join(REPO, "model", "ffd_model.bin"))
    lines = open(os.path.join(REF, "output", "errors.txt")).read().splitlines(True)
    fx = load_fixtures()
    pins, others = [], []
    for k, (name, img, box, parts) in enumerate(zip(fx["names"], fx["images"], fx["boxes"], fx["parts"])):
        f, _ = oracle.analyze_face(img, tuple(int(v) for v in box), threads=8)
        line = fe.format_errors([fe.landmark_errors(parts, f["points"])])
        hits = [i + 1 for i, l in enumerate(lines) if l == line]
        if hits:
            pins.append({"fixture": k, "name": str(name), "box": [int(v) for v in box], "errors_txt_line": hits[0],
                         "line": line, "oracle_points": np.asarray(f["points"]).tolist()})
        else:
            tok = line.split()
            best = max(sum(a == b for a, b in zip(l.split(), tok)) for l in lines)
            others.append({"fixture": k, "name": str(name), "best_entry_overlap": int(best)})
    doc = {
        "source": "/root/reference/output/errors.txt (eval_ffd.cpp:102-121), 1326 LFW test faces",
        "method": "tests/golden/make_reference_pins.py: oracle.analyze_face on the fixture face with its "
                  "annotated box, eval.format_errors, exact line lookup",
        "pins": pins,
        "not_in_errors_txt": others,
    }
    with open(OUT, "w") as fh:
        json.dump(doc, fh, indent=1)
    print("wrote", OUT, "pins:", [(p["name"], p["errors_txt_line"]) for p in pins])


if __name__ == "__main__":
    sys.exit(main())
