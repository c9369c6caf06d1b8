"""The header-only C++ drop-in (include/FaceForest.hpp) through examples/analyze_face.cpp:
the reference's analyzeFace call contract from C++ (eval_ffd.cpp:89, demo.cpp:149)."""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "examples", "build", "analyze_face")


def _run(model_path, img, box, tmp_path):
    path = tmp_path / "img.bgr"
    np.ascontiguousarray(img).tofile(path)
    h, w = img.shape[:2]
    return subprocess.run([EXE, model_path, str(path), str(w), str(h)] + [str(int(v)) for v in box],
                          capture_output=True, text=True, timeout=300)


def test_shim_reports_missing_device(model_path, fixtures, tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    assert os.path.exists(EXE), "run `make` (__graft_entry__.build())"
    r = _run(model_path, fixtures["images"][0], fixtures["boxes"][0], tmp_path)
    assert r.returncode == 3 and "no HIP device" in r.stderr


@pytest.mark.gpu
def test_shim_matches_python_engine(model_path, fixtures, engine, tmp_path):
    for i in (0, 7):
        img, box = fixtures["images"][i], tuple(int(v) for v in fixtures["boxes"][i])
        r = _run(model_path, img, box, tmp_path)
        assert r.returncode == 0, r.stderr
        vals = r.stdout.split()
        face = engine.analyzeFace(img, box)
        assert np.float32(float(vals[0])) == np.float32(face.headpose)
        assert np.array_equal(np.array(vals[1:], np.int32).reshape(10, 2), face.ffd_cordinates)


@pytest.mark.gpu
def test_shim_estimators_and_forest(model_path, fixtures, engine, oracle_mod, tmp_path):
    """ImageSample + static estimateHeadPose / estimateFacialFeatures + Forest<HeadPoseSample>::evaluateMT
    from C++ (examples/estimate.cpp) against the Python engine and the oracle."""
    img, box = fixtures["images"][5], tuple(int(v) for v in fixtures["boxes"][5])
    engine.analyzeFace(img, box)
    gray = engine.trace(0, box[2], box[3])["face"]
    h, w = gray.shape
    path = tmp_path / "face.gray"
    np.ascontiguousarray(gray).tofile(path)
    region, pose_bin = (4, 2, 115, 120), 2
    exe = os.path.join(REPO, "examples", "build", "estimate")
    r = subprocess.run([exe, model_path, str(path), str(w), str(h)] + [str(v) for v in region] + [str(pose_bin)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    ch = oracle_mod.channels(gray)
    hp, var = oracle_mod.estimate_headpose(ch, region)
    got_hp, got_var = (float(v) for v in lines[0].split())
    assert np.float32(got_hp) == np.float32(hp) and np.float32(got_var) == np.float32(var)
    pts = np.array(lines[1].split(), np.int32).reshape(10, 2)
    assert np.array_equal(pts, oracle_mod.estimate_facial_features(ch, region, range(pose_bin * 20, pose_bin * 20 + 20)))
    leaves = np.array(lines[2].split(), np.int32)
    import face_alignment_cvpr_2012_amd as ffd
    want = ffd.Forest(engine, ffd.FOREST_HEADPOSE).evaluate(ch, [region[:2]], list(range(15)))[0]
    assert np.array_equal(leaves, want)
    # Forest<MPSample>::evaluateMT(const MPSample*, MPLeaf**): the reference's Leaf members
    from face_alignment_cvpr_2012_amd import model as fm
    m = fm.load(model_path)
    ids = ffd.Forest(engine, ffd.FOREST_FFD).evaluate(ch, [region[:2]], list(range(pose_bin * 20, pose_bin * 20 + 20)))[0]
    got = np.array(lines[3].split(), np.float64).reshape(20, 4)
    np.testing.assert_array_equal(got[:, 0], m["mp.leaf_n"][ids])
    np.testing.assert_array_equal(got[:, 1].astype(np.float32), m["mp.leaf_fg"][ids])
    np.testing.assert_array_equal(got[:, 2:].astype(np.int32), m["mp.leaf_offset"][ids][:, 0, :])

    # the static estimators honour their options argument (the engine keeps its defaults)
    extra = ["hp_min_fg=0.6", "hp_step=5", "mp_min_pf=0.3", "mp_max_var=20", "mp_parts=8", "mp_step=4"]
    r = subprocess.run([exe, model_path, str(path), str(w), str(h)] + [str(v) for v in region] + [str(pose_bin)] + extra,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    oracle_mod.set_options(hp_min_fg=0.6, hp_step=5, mp_min_pf=0.3, mp_max_var=20.0, mp_num_parts=8, mp_step_x=4,
                           mp_step_y=4)
    try:
        hp, var = oracle_mod.estimate_headpose(ch, region)
        want_pts = oracle_mod.estimate_facial_features(ch, region, range(pose_bin * 20, pose_bin * 20 + 20))
    finally:
        oracle_mod.reset_options()
    got_hp, got_var = (float(v) for v in lines[0].split())
    assert np.float32(got_hp) == np.float32(hp) and np.float32(got_var) == np.float32(var)
    pts = np.array(lines[1].split(), np.int32).reshape(8, 2)
    assert np.array_equal(pts, want_pts[:8])


@pytest.mark.gpu
def test_shim_analyze_image_detects(model_path, fixtures, engine, tmp_path):
    """analyzeImage(img, faces) from C++: the GPU Haar detector then analyzeFace, equal to the Python API."""
    img = fixtures["images"][9]
    path = tmp_path / "img.bgr"
    np.ascontiguousarray(img).tofile(path)
    h, w = img.shape[:2]
    r = subprocess.run([EXE, model_path, str(path), str(w), str(h)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = [ln.split() for ln in r.stdout.strip().splitlines()]
    faces = engine.analyzeImage(img)
    assert len(lines) == len(faces) == 1
    for ln, f in zip(lines, faces):
        assert tuple(int(v) for v in ln[:4]) == f.bbox
        assert np.float32(float(ln[4])) == np.float32(f.headpose)
        assert np.array_equal(np.array(ln[5:], np.int32).reshape(10, 2), f.ffd_cordinates)


def _evaluate_mt(model_path, gray, trees, tmp_path, env=None):
    import json
    path = tmp_path / "face_mt.gray"
    np.ascontiguousarray(gray).tofile(path)
    h, w = gray.shape
    exe = os.path.join(REPO, "examples", "build", "evaluate_mt")
    r = subprocess.run([exe, model_path, str(path), str(w), str(h)] + [str(int(t)) for t in trees],
                       capture_output=True, text=True, timeout=300, env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("k", [0, 11])
def test_shim_evaluate_mt_per_patch_pattern(model_path, fixtures, oracle_mod, tmp_path, k):
    """getFacialFeaturesVotesMT's call pattern from C++ (examples/evaluate_mt.cpp): ImageSample(cv::Mat, features,
    true), the per-face Forest<MPSample> composed by addTree(jungle[i].getTree(j)), 1,024 evaluateMT(const
    MPSample*, MPLeaf**) calls on copies of the forest, the reference's vote filter over the Leaf* members and
    MeanShift::shift per landmark.  Leaf ordinals, vote counts, the MeanShift modes (bitwise) and the landmarks
    equal the oracle's analyzeFace of the same face and trees."""
    import zlib
    img, box = fixtures["images"][k], tuple(int(v) for v in fixtures["boxes"][k])
    ref, tr = oracle_mod.analyze_face(img, box, threads=8, trace=True)
    d = _evaluate_mt(model_path, tr["face"], tr["trees"], tmp_path)
    assert d["patches"] == tr["mp_leaves"].shape[0] and d["trees"] == len(tr["trees"])
    assert d["leaf_crc"] == zlib.crc32(np.ascontiguousarray(tr["mp_leaves"], np.int32).tobytes())
    assert d["vote_counts"] == [int(v) for v in tr["vote_counts"]]
    modes = np.array(d["modes"], np.float32)
    assert np.array_equal(modes.view(np.uint32), np.asarray(tr["ms_mean"], np.float32).view(np.uint32))
    assert np.array_equal(np.array(d["points"], np.int32), np.rint(tr["ms_mean"]).astype(np.int32))
    # the per-call cost after the grid evaluation is a host-side lookup; report it
    assert d["other_calls_mean_us"] < 100.0, d
    print("evaluate_mt timings:", {key: d[key] for key in ("sample_ms", "first_call_ms", "other_calls_mean_us",
                                                           "all_calls_ms", "vote_filter_ms", "meanshift_ms")})


@pytest.mark.gpu
@pytest.mark.parametrize("shared", [0, 1])
def test_shim_evaluate_mt_threads_share_engine(model_path, fixtures, oracle_mod, tmp_path, shared):
    """Pool threads on one engine (face_utils.cpp:210-216, 267-274 run evaluateMT from a thread pool): 6 threads,
    each with its own ImageSample, walk every patch four times, each with its own Forest (separate caches) or with
    copies of one Forest (one cache: a thread replaces the cached grid while the others still read the grid they
    hold without a lock); each thread's leaf CRC equals the oracle's."""
    import zlib
    img, box = fixtures["images"][2], tuple(int(v) for v in fixtures["boxes"][2])
    ref, tr = oracle_mod.analyze_face(img, box, threads=8, trace=True)
    d = _evaluate_mt(model_path, tr["face"], tr["trees"], tmp_path,
                     env={"FFD_EVAL_THREADS": "6", "FFD_EVAL_REPS": "1", "FFD_EVAL_SHARED": str(shared)})
    want = zlib.crc32(np.ascontiguousarray(tr["mp_leaves"], np.int32).tobytes())
    assert d["leaf_crc"] == want
    assert d["thread_errors"] == 0 and d["thread_crcs"] == [want] * 6, d


@pytest.mark.gpu
def test_sample_eval_leaves_matches_oracle(model_path, fixtures, engine, oracle_mod):
    """ffd_sample_eval_leaves / ffd_sample_eval_grid on a device-resident sample (off-grid patches, long lists,
    head-pose and FFD trees) against the oracle's walks; the sample's channels read back equal the oracle's."""
    import face_alignment_cvpr_2012_amd as ffd
    img, box = fixtures["images"][3], tuple(int(v) for v in fixtures["boxes"][3])
    ref, tr = oracle_mod.analyze_face(img, box, threads=8, trace=True)
    gray = tr["face"]
    with ffd.ImageSample(engine, gray) as s:
        assert np.array_equal(s.channels(), tr["channels"])
        # the FFD grid equals the oracle's leaves in the reference order
        h, w = gray.shape
        nx, ny = len(range(0, w - 31, 3)), len(range(0, h - 31, 3))
        got = s.eval_grid(ffd.FOREST_FFD, 0, 0, 3, nx, ny, tr["trees"])
        assert np.array_equal(got, tr["mp_leaves"].reshape(nx * ny, -1))
        # patch lists: inline (<= 16) and uploaded, arbitrary positions; the head-pose forest
        rng = np.random.default_rng(5)
        for n in (1, 7, 16, 17, 300):
            xy = np.stack([rng.integers(0, w - 31 + 1, n), rng.integers(0, h - 31 + 1, n)], 1).astype(np.int32)
            want = oracle_mod.eval_patches(tr["channels"], xy, ffd.FOREST_HEADPOSE, list(range(15)))
            assert np.array_equal(s.eval_leaves(ffd.FOREST_HEADPOSE, xy, list(range(15))), want)


@pytest.mark.gpu
def test_tall_sample_float_integrals_match_oracle(fixtures, engine, oracle_mod):
    """A sample whose integrals pass 2^24 (a 125 x 1500 face: 255 W H >= 2^24, where the reference's CV_32F
    integrals round) keeps the rounded values and is walked with the float rectangle means: its channels read
    back, the FFD grid, patch lists, the whole-sample and sub-region estimates, a sample made from those
    channels and ffd_forest_eval_leaves on them all equal the oracle."""
    import face_alignment_cvpr_2012_amd as ffd
    img, box = fixtures["images"][0], (100, 5, 20, 240)
    ref, tr = oracle_mod.analyze_face(img, box, threads=16, trace=True)
    gray, ch = tr["face"], tr["channels"]
    h, w = gray.shape
    assert 255 * w * h >= 1 << 24 and ch.max() >= 1 << 24
    rng = np.random.default_rng(9)
    xy = np.stack([rng.integers(0, w - 31 + 1, 300), rng.integers(0, h - 31 + 1, 300)], 1).astype(np.int32)
    want_hp = oracle_mod.eval_patches(ch, xy, ffd.FOREST_HEADPOSE, list(range(15)))
    want_mp = oracle_mod.eval_patches(ch, xy[:12], ffd.FOREST_FFD, tr["trees"])
    assert np.array_equal(ffd.Forest(engine, ffd.FOREST_HEADPOSE).evaluate(ch, xy, list(range(15))), want_hp)
    for s in (ffd.ImageSample(engine, gray), ffd.ImageSample(engine, channels=ch)):
        with s:
            assert np.array_equal(s.channels(), ch)
            nx, ny = len(range(0, w - 31, 3)), len(range(0, h - 31, 3))
            got = s.eval_grid(ffd.FOREST_FFD, 0, 0, 3, nx, ny, tr["trees"])
            assert np.array_equal(got, tr["mp_leaves"].reshape(nx * ny, -1))
            assert np.array_equal(s.eval_leaves(ffd.FOREST_HEADPOSE, xy, list(range(15))), want_hp)
            assert np.array_equal(s.eval_leaves(ffd.FOREST_FFD, xy[:12], tr["trees"]), want_mp)
            hp, var = s.estimateHeadPose()
            assert np.float32(hp) == np.float32(ref["headpose"])
            assert np.array_equal(s.estimateFacialFeatures(None, tr["trees"]), np.rint(tr["ms_mean"]).astype(np.int32))
            for region in ((3, 200, 110, 700), (0, 900, 125, 600)):
                o = oracle_mod.estimate_headpose(ch, region)
                g = s.estimateHeadPose(region)
                assert np.float32(g[0]) == np.float32(o[0]) and np.float32(g[1]) == np.float32(o[1]), region
                assert np.array_equal(s.estimateFacialFeatures(region, tr["trees"]),
                                      oracle_mod.estimate_facial_features(ch, region, tr["trees"])), region
