"""Accuracy harness: the reference's eval_ffd metric and report.

* ``inter_ocular_distance`` — getInterOccularDist (src/eval_ffd.cpp:33-46): distance between the
  mid-points of landmarks (0, 1) and (6, 7), in float as the reference's cv::Point2f.
* ``landmark_errors`` — evalForest's per-face errors (src/eval_ffd.cpp:102-108): cv::norm of the
  integer landmark difference divided by the inter-ocular distance.
* ``format_errors`` / ``parse_errors`` — the output/errors.txt format (src/eval_ffd.cpp:112-121):
  one face per line, values in C++ ostream default format (6 significant digits) each followed by
  a space.
* ``report`` — output/generate_report.m:7-10: per-landmark mean error and accuracy (% of faces
  with error < 0.1 IOD), plus the all-landmark aggregates quoted in BASELINE.md.

CLI (GPU): ``python -m face_alignment_cvpr_2012_amd.eval [--out errors.txt]`` runs the engine on
the 20 annotated faces the reference ships (tests/golden/faces.npz) and prints the report.
"""
import argparse
import math
import sys

import numpy as np

LANDMARK_NAMES = ("left eye (l)", "left eye (r)", "mouth (l)", "mouth (r)", "mouth (b)", "mouth (t)",
                  "right eye (l)", "right eye (r)", "nose (l)", "nose (r)")  # generate_report.m:13-15
IOD_THRESHOLD = 0.1                                                          # generate_report.m:9


def inter_ocular_distance(parts):
    p = np.asarray(parts, np.float32)
    two = np.float32(2.0)
    lx, ly = (p[0, 0] + p[1, 0]) / two, (p[0, 1] + p[1, 1]) / two
    rx, ry = (p[6, 0] + p[7, 0]) / two, (p[6, 1] + p[7, 1]) / two
    dx, dy = float(np.float32(lx - rx)), float(np.float32(ly - ry))
    return np.float32(math.sqrt(dx * dx + dy * dy))


def landmark_errors(parts, predicted):
    """parts, predicted: 10 x 2 integer landmarks in the same (box-relative) frame."""
    iod = inter_ocular_distance(parts)
    out = []
    for (gx, gy), (px, py) in zip(np.asarray(parts, np.int64), np.asarray(predicted, np.int64)):
        d = np.float32(math.sqrt(float((gx - px) ** 2 + (gy - py) ** 2)))
        out.append(np.float32(d / iod))
    return np.array(out, np.float32)


def _cpp_float(v):
    """C++ `ostream << float` with the default precision (6 significant digits, %g)."""
    return "%g" % float(v)


def format_errors(errors):
    return "".join("".join(_cpp_float(v) + " " for v in row) + "\n" for row in errors)


def parse_errors(text):
    rows = [line.split() for line in text.splitlines() if line.strip()]
    return np.array([[float(v) for v in r] for r in rows], np.float64)


def report(errors):
    e = np.asarray(errors, np.float64)
    per_mean = e.mean(axis=0)
    per_acc = (e < IOD_THRESHOLD).sum(axis=0) / e.shape[0] * 100.0
    return {
        "faces": int(e.shape[0]),
        "mean_error": float(e.mean()),
        "median_error": float(np.median(e)),
        "accuracy_pct": float((e < IOD_THRESHOLD).mean() * 100.0),
        "per_landmark_mean": [float(v) for v in per_mean],
        "per_landmark_accuracy_pct": [float(v) for v in per_acc],
    }


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--out", default=None, help="write errors.txt here")
    ap.add_argument("--device", type=int, default=0)
    args = ap.parse_args(argv)

    import face_alignment_cvpr_2012_amd as ffd
    from face_alignment_cvpr_2012_amd.synthetic import load_fixtures

    fx = load_fixtures()
    boxes = [tuple(int(v) for v in b) for b in fx["boxes"]]
    with ffd.FaceForest(ffd.FaceForestOptions(device=args.device)) as ff:
        faces = ff.analyzeFaces(list(fx["images"]), boxes)
    errors = [landmark_errors(p, f.ffd_cordinates) for p, f in zip(fx["parts"], faces)]
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(format_errors(errors))
    r = report(errors)
    print(f"faces {r['faces']}  mean IOD error {r['mean_error']:.4f}  median {r['median_error']:.4f}  "
          f"accuracy(<{IOD_THRESHOLD}) {r['accuracy_pct']:.1f}%")
    for name, m, a in zip(LANDMARK_NAMES, r["per_landmark_mean"], r["per_landmark_accuracy_pct"]):
        print(f"  {name:14s} {m:.4f}  {a:5.1f}%")
    return 0


if __name__ == "__main__":
    sys.exit(main())
