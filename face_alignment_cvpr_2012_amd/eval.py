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

* ``eval_forest`` — evalForest (src/eval_ffd.cpp:57-122): every test annotation's image loaded
  (loadImage; faces whose image does not load are skipped, as the reference's ``continue``),
  ``analyzeFace(img, annotation.bbox)``, the errors in the test set's order (pose buckets 0..4, file
  order inside a bucket).  The engine runs the faces as batches (one analyzeFace per face gives the
  same records: tests/test_golden.py).
* ``run_eval`` — eval_ffd's main (src/eval_ffd.cpp:133-179): config files, annotations, the pose-bucketed
  90 / 10 split (config.split_by_pose), evalForest, errors.txt.

CLI (GPU): ``python -m face_alignment_cvpr_2012_amd.eval`` runs eval_ffd on the 20 annotated faces the
reference ships (tests/golden/index_random_subset.txt with the images pre-decoded in
tests/golden/faces.npz: the split's 5 test faces); ``--all`` scores all 20; ``--annotations FILE
[--images DIR | --arrays NPZ]`` runs it on any annotation set in the reference's format (e.g. LFW's
lfw_ffd_ann.txt, decoded with Pillow); ``--out errors.txt`` writes the reference's errors.txt.
"""
import os
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


def eval_forest(analyzer, test_buckets, load_image, batch=1024, log=None):
    """evalForest (src/eval_ffd.cpp:57-122).  analyzer: an object with analyzeFaces(images, boxes,
    box_img) (the engine's FaceForest) or analyzeFace(img, bbox); test_buckets: the test split's pose
    buckets; load_image: name -> BGR array or None.  Returns (errors, evaluated annotations)."""
    annotations = [a for b in test_buckets for a in b]
    done, errors = [], []
    pend_imgs, pend_idx, pend_ann = [], {}, []

    def flush():
        if not pend_ann:
            return
        boxes = [tuple(int(v) for v in a.bbox) for a, _ in pend_ann]
        box_img = np.array([k for _, k in pend_ann], np.int32)
        if hasattr(analyzer, "analyzeFaces"):
            faces = analyzer.analyzeFaces(pend_imgs, boxes, box_img)
        else:
            faces = [analyzer.analyzeFace(pend_imgs[k], b) for b, k in zip(boxes, box_img)]
        for (a, _), f in zip(pend_ann, faces):
            errors.append(landmark_errors(a.parts, f.ffd_cordinates))
            done.append(a)
        pend_imgs.clear()
        pend_idx.clear()
        pend_ann.clear()

    for a in annotations:
        if a.url not in pend_idx:
            img = load_image(a.url)
            if img is None or img.size == 0:
                if log:
                    log(f"Could not load: {a.url}")  # eval_ffd.cpp:81-85
                continue
            pend_idx[a.url] = len(pend_imgs)
            pend_imgs.append(img)
        pend_ann.append((a, pend_idx[a.url]))
        if len(pend_ann) >= batch:
            flush()
    flush()
    return errors, done


def run_eval(analyzer, annotations_path, load_image=None, out_path="output/errors.txt", all_faces=False, log=None):
    """eval_ffd main (src/eval_ffd.cpp:133-179) from an annotation file: the pose-bucketed 90 / 10
    split, evalForest over the test part (or every annotation with all_faces), errors.txt."""
    from face_alignment_cvpr_2012_amd import config

    ok, anns = config.load_annotations(annotations_path)
    if not ok:
        raise FileNotFoundError(annotations_path)
    _, test = config.split_by_pose(anns)
    if all_faces:
        test = [anns]
    if load_image is None:
        load_image = config.ImageStore(config.image_dir(annotations_path))
    errors, done = eval_forest(analyzer, test, load_image, log=log)
    if out_path:
        d = os.path.dirname(out_path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(out_path, "w") as fh:
            fh.write(format_errors(errors))
    return errors, done


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ap.add_argument("--annotations", default=os.path.join(here, "tests", "golden", "index_random_subset.txt"),
                    help="annotation file in the reference's format (loadAnnotations)")
    ap.add_argument("--images", default=None, help="image directory (default: the annotation file's)")
    ap.add_argument("--arrays", default=None, help=".npz of pre-decoded BGR images (names + images, or name -> array)")
    ap.add_argument("--all", action="store_true", help="score every annotation, not only the 10 %% test split")
    ap.add_argument("--out", default=None, help="write errors.txt here")
    ap.add_argument("--device", type=int, default=0)
    args = ap.parse_args(argv)

    import face_alignment_cvpr_2012_amd as ffd
    from face_alignment_cvpr_2012_amd import config

    arrays = args.arrays
    if arrays is None and args.images is None and args.annotations.endswith(os.path.join("golden", "index_random_subset.txt")):
        arrays = os.path.join(os.path.dirname(args.annotations), "faces.npz")
    store = config.ImageStore(args.images + "/" if args.images else config.image_dir(args.annotations), arrays)
    with ffd.FaceForest(ffd.FaceForestOptions(device=args.device)) as ff:
        errors, done = run_eval(ff, args.annotations, store, out_path=args.out, all_faces=args.all,
                                log=lambda m: print(m, file=sys.stderr))
    if not errors:
        print("no face evaluated")
        return 1
    r = report(errors)
    print(f"faces {r['faces']}  mean IOD error {r['mean_error']:.4f}  median {r['median_error']:.4f}  "
          f"accuracy(<{IOD_THRESHOLD}) {r['accuracy_pct']:.1f}%")
    for name, m, a in zip(LANDMARK_NAMES, r["per_landmark_mean"], r["per_landmark_accuracy_pct"]):
        print(f"  {name:14s} {m:.4f}  {a:5.1f}%")
    return 0


if __name__ == "__main__":
    sys.exit(main())
