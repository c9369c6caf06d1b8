"""Leaf-level A/B check of two libffd.so builds on a bench workload (GPU).

usage: FFD_LIBRARY=build/X/libffd.so python tools/leaf_ab.py --out gpurun_out/x.npz [--workload c2] [--faces 4096]
       python tools/leaf_ab.py --compare gpurun_out/a.npz gpurun_out/b.npz

Runs analyzeFaces once on the workload and records, per face, the head pose, the landmarks and CRC-32s of the
head-pose and FFD leaf ordinals (ffd_get_trace); --compare reports the faces whose records differ.  Used to
keep a traversal rewrite bit-exact with the build it replaces on every face of the batch, beside the oracle
parity tests (which cover fewer faces).
"""
import argparse
import ctypes
import os
import sys
import zlib

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def record(workload, faces):
    import bench
    import face_alignment_cvpr_2012_amd as fa
    wl = bench.make_workload(workload, 0, 1, faces, 64)
    os.environ["FFD_HOST_CHUNK"] = str(faces)  # one chunk: every face's trace stays readable
    mp = fa.MultiPartEstimatorOption(step_size=wl.mp_steps[0], step_size_y=wl.mp_steps[1])
    ff = fa.FaceForest(fa.FaceForestOptions(model_path=wl.model, mp_option=mp, max_chunk_faces=faces))
    res = ff.analyzeFaces(wl.images, wl.boxes, wl.box_img)
    n = len(res)
    hp = np.array([r.headpose for r in res], np.float32)
    pts = np.array([r.ffd_cordinates for r in res], np.int32).reshape(n, -1)
    crc = np.zeros((n, 2), np.uint32)
    for i in range(n):  # the leaf buffers only (no face / channel downloads)
        b = wl.boxes[i]
        fw, fh, nhp, nmp = ff.geometry(b[2], b[3])
        hl, ml = np.zeros((nhp, 15), np.int32), np.zeros(nmp * fa.MAX_TREES, np.int32)
        tr = fa._Trace(None, None, hl.ctypes.data, ml.ctypes.data, None, None, None, None)
        fa._check(fa.lib().ffd_get_trace(ff.handle, i, ctypes.byref(tr)), ff.handle)
        crc[i, 0] = zlib.crc32(hl.tobytes())
        crc[i, 1] = zlib.crc32(ml.tobytes())
    return dict(hp=hp, pts=pts, crc=crc)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--faces", type=int, default=4096)
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.compare:
        x, y = (np.load(p) for p in a.compare)
        bad = ((x["hp"].view(np.uint32) != y["hp"].view(np.uint32)) | (x["pts"] != y["pts"]).any(axis=1) |
               (x["crc"] != y["crc"]).any(axis=1))
        print(f"faces {len(bad)} differing {int(bad.sum())} (hp leaves {int((x['crc'][:, 0] != y['crc'][:, 0]).sum())},"
              f" ffd leaves {int((x['crc'][:, 1] != y['crc'][:, 1]).sum())})", flush=True)
        if bad.any():
            print("first:", np.nonzero(bad)[0][:10].tolist())
        sys.exit(1 if bad.any() else 0)
    d = record(a.workload, a.faces)
    np.savez(a.out, **d)
    print(f"{a.out}: {len(d['hp'])} faces", flush=True)


if __name__ == "__main__":
    main()
