"""The drop-in boundary proven from C++: tests/native/boundary_test.cpp is compiled by g++
against include/orbx*.h alone and linked to liborbx.so, as the reference's C++ would bind it
(include/ORBextractor.h:45-111, include/ORBmatcher.h:37-128).

* CPU: the program's sizeof / offsetof of every ABI struct equal the Python ctypes / numpy
  mirrors (features.py, matcher.py, _lib.py, oracle/matcher.py), so a layout drift fails a test;
  its static_asserts pin orbx_keypoint to cv::KeyPoint's 28-byte layout at compile time.
* GPU: the INTEGRATION.md sequence (two extraction std::threads, Frame.cc:89-92; stereo;
  SearchByBoW; SearchForTriangulation) on a KITTI fixture pair: outputs equal the committed
  golden digests (tests/golden/fixtures.json) and the restated matchers.
"""
import ctypes
import hashlib
import json
import pathlib
import subprocess

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
GOLDEN = json.loads((ROOT / "tests" / "golden" / "fixtures.json").read_text())


@pytest.fixture(scope="module")
def boundary_bin(orbx_lib):
    from my_orb_slam2_amd import build as b
    return b.build_boundary_test()


def _ctypes_layout(cls):
    return {name: [getattr(cls, name).offset, getattr(cls, name).size] for name, _ in cls._fields_}


def _dtype_layout(dt):
    return {name: [dt.fields[name][1], dt.fields[name][0].itemsize] for name in dt.names}


def test_struct_layouts_match_python_mirrors(boundary_bin):
    from my_orb_slam2_amd._lib import KEYPOINT_DTYPE, BatchView, ExtractorParams
    from my_orb_slam2_amd.features import PROJ_QUERY_DTYPE, FeatureSetC
    from my_orb_slam2_amd.kfdb import KfdbParams
    from my_orb_slam2_amd.matcher import KfDbC, MatcherParams
    import oracle
    from oracle import matcher as om
    out = subprocess.run([str(boundary_bin), "layout"], check=True, capture_output=True,
                         text=True, timeout=60).stdout
    c = json.loads(out)
    mirrors = {
        "orbx_keypoint": [_dtype_layout(KEYPOINT_DTYPE), _dtype_layout(oracle.KEYPOINT_DTYPE)],
        "orbx_extractor_params": [_ctypes_layout(ExtractorParams)],
        "orbx_batch_view": [_ctypes_layout(BatchView)],
        "orbx_featureset": [_ctypes_layout(FeatureSetC), _ctypes_layout(om._FeatC)],
        "orbx_matcher_params": [_ctypes_layout(MatcherParams)],
        "orbx_kf_db": [_ctypes_layout(KfDbC)],
        "orbx_proj_query": [_dtype_layout(PROJ_QUERY_DTYPE)],
        "orbx_kfdb_params": [_ctypes_layout(KfdbParams)],
    }
    sizes = {"orbx_keypoint": [KEYPOINT_DTYPE.itemsize, oracle.KEYPOINT_DTYPE.itemsize],
             "orbx_extractor_params": [ctypes.sizeof(ExtractorParams)],
             "orbx_batch_view": [ctypes.sizeof(BatchView)],
             "orbx_featureset": [ctypes.sizeof(FeatureSetC), ctypes.sizeof(om._FeatC)],
             "orbx_matcher_params": [ctypes.sizeof(MatcherParams)],
             "orbx_kf_db": [ctypes.sizeof(KfDbC)],
             "orbx_proj_query": [PROJ_QUERY_DTYPE.itemsize],
             "orbx_kfdb_params": [ctypes.sizeof(KfdbParams)]}
    for name, lays in mirrors.items():
        assert name in c, name
        for lay in lays:
            assert lay == c[name]["fields"], f"{name}: python {lay} vs C {c[name]['fields']}"
        for sz in sizes[name]:
            assert sz == c[name]["size"], f"{name}: size {sz} vs C {c[name]['size']}"
    assert c["orbx_keypoint"]["size"] == 28


def _sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1])
def test_cpp_dropin_sequence(boundary_bin, oracle_mod, gpu, tmp_path, seed):
    from oracle import matcher as om
    from my_orb_slam2_amd import synth
    from my_orb_slam2_amd._lib import KEYPOINT_DTYPE
    from my_orb_slam2_amd.features import FeatureSet, feature_vector
    g = GOLDEN[f"kitti_stereo_seed{seed}"]
    L, R = synth.stereo_pair(seed)
    assert [_sha(L.tobytes()), _sha(R.tobytes())] == g["input_sha256"]
    H, W = L.shape
    (tmp_path / "left.raw").write_bytes(L.tobytes())
    (tmp_path / "right.raw").write_bytes(R.tobytes())
    # a rectified pair: epipolar lines are rows (F12 = [t]_x for t along x), epipole at infinity
    F12 = np.array([[0, 0, 0], [0, 0, -1], [0, 1, 0]], np.float32)
    ex, ey = 1.0e7, 0.0
    (tmp_path / "params.txt").write_text(
        f"{W} {H} {g['params'][0]} {g['mbf']!r} {g['mb']!r} {ex!r} {ey!r} " +
        " ".join(repr(float(v)) for v in F12.reshape(-1)))
    r = subprocess.run([str(boundary_bin), "run", str(tmp_path)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    rd = lambda name: (tmp_path / name).read_bytes()
    n = int(np.frombuffer(rd("n.bin"), np.int32)[0])
    nr = int(np.frombuffer(rd("nr.bin"), np.int32)[0])
    assert (n, nr) == (g["n_left"], g["n_right"])
    assert int(np.frombuffer(rd("nvalid.bin"), np.int32)[0]) == g["n_valid"]
    for key, fname in (("kps_left", "kps_left.bin"), ("desc_left", "desc_left.bin"),
                       ("kps_right", "kps_right.bin"), ("desc_right", "desc_right.bin"),
                       ("uRight", "uRight.bin"), ("depth", "depth.bin")):
        assert _sha(rd(fname)) == g["sha256"][key], key
    # the matchers on the views the program extracted, against the restatement
    kl = np.frombuffer(rd("kps_left.bin"), KEYPOINT_DTYPE)
    kr = np.frombuffer(rd("kps_right.bin"), KEYPOINT_DTYPE)
    dl = np.frombuffer(rd("desc_left.bin"), np.uint8).reshape(-1, 32)
    dr = np.frombuffer(rd("desc_right.bin"), np.uint8).reshape(-1, 32)
    F = FeatureSet(kl.copy(), dl.copy(), None, feature_vector(np.zeros(n)), None)
    KF = FeatureSet(kr.copy(), dr.copy(), None, feature_vector(np.zeros(nr)), None)
    bow = np.frombuffer(rd("bow.bin"), np.int32)
    n_o, m_o = om.search_by_bow_kf_frame(KF, np.ones(nr, bool), F, 0.75, True)
    assert bow[0] == n_o and n_o > 0
    np.testing.assert_array_equal(bow[1:], m_o)
    tri = np.frombuffer(rd("tri.bin"), np.int32)
    s, s2, _ = synth.scale_tables()
    t_o, p_o = om.search_for_triangulation(F, np.zeros(n, bool), KF, np.zeros(nr, bool), F12,
                                           np.array([ex, ey], np.float32), s2, s, False, False)
    assert tri[0] == t_o and t_o > 0
    np.testing.assert_array_equal(tri[1:].reshape(-1, 2), p_o)


@pytest.mark.gpu
def test_cpp_tum_mode_parity(boundary_bin, oracle_mod, gpu, tmp_path):
    """bench.py --workload tum's own loop (boundary_test `tum`, configs[0]: extraction,
    ComputeBoW with the synthetic k=10 L=5 vocabulary at levelsup 3, ORBmatcher(0.7, true)
    .SearchByBoW(KF, F)) at its bench geometry (640x480, 1000 features, the same seeds): the
    dumped keyframe / frame features, BoW / FeatureVectors and matches equal the restatement's
    on the same images."""
    import bench
    import oracle
    from oracle import matcher as om
    from my_orb_slam2_amd import synth
    from my_orb_slam2_amd._lib import KEYPOINT_DTYPE
    from my_orb_slam2_amd.features import FeatureSet, FeatureVector
    P, levelsup = 3, 3
    W, H, nfeat = bench.TUM_W, bench.TUM_H, bench.TUM_NFEAT
    pairs = [synth.stereo_pair(3000 + i, W, H) for i in range(P)]
    voc = tmp_path / "voc.txt"
    synth.write_vocabulary(str(voc), k=10, L=5, seed=11)
    for i, (L, R) in enumerate(pairs):
        L.tofile(tmp_path / f"pair_{i}_left.raw")
        R.tofile(tmp_path / f"pair_{i}_right.raw")
    (tmp_path / "params.txt").write_text(f"{W} {H} {nfeat} {P} {levelsup} {voc}\n")
    dump = tmp_path / "dump"
    dump.mkdir()
    r = subprocess.run([str(boundary_bin), "tum", str(tmp_path), "2", str(P), str(dump)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["mean_keypoints"] > 0.9 * nfeat and res["mean_bow_matches"] > 0
    ov = om.OracleVocabulary(str(voc))
    ox = oracle.OracleExtractor(nfeat, 1.2, 8, 20, 7)

    def check(prefix, img):
        rd = lambda s, dt: np.fromfile(dump / f"{prefix}_{s}.bin", dt)
        k = rd("kps", KEYPOINT_DTYPE)
        d = rd("desc", np.uint8).reshape(-1, 32)
        ko, do = ox(img)
        np.testing.assert_array_equal(k.view(np.uint8), np.ascontiguousarray(ko).view(np.uint8))
        np.testing.assert_array_equal(d, do)
        _, _, (bw, bv), (fn, fo, ff) = ov.transform(do, levelsup)
        np.testing.assert_array_equal(rd("bow_w", np.uint32), bw)
        np.testing.assert_array_equal(rd("bow_v", np.float64), bv)
        np.testing.assert_array_equal(rd("fv_node", np.uint32), fn)
        np.testing.assert_array_equal(rd("fv_off", np.int32), fo)
        np.testing.assert_array_equal(rd("fv_feat", np.int32), ff)
        return FeatureSet(ko, do, None, FeatureVector(fn, fo, ff), None)

    total = 0
    for i, (L, R) in enumerate(pairs):
        kf = check(f"kf_{i}", L)
        fr = check(f"frame_{i}", R)
        valid = np.fromfile(dump / f"kf_{i}_valid.bin", np.uint8).astype(bool)
        assert len(valid) == len(kf.keys) and 0.75 < valid.mean() < 0.95
        n_o, m_o = om.search_by_bow_kf_frame(kf, valid, fr, 0.7, True)
        assert int(np.fromfile(dump / f"frame_{i}_nm.bin", np.int32)[0]) == n_o
        np.testing.assert_array_equal(np.fromfile(dump / f"frame_{i}_matches.bin", np.int32), m_o)
        total += n_o
    assert total > 0
