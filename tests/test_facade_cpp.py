"""The drop-in facade itself, compiled: integration/ORBextractor.h (ORB_SLAM2::ORBextractor,
include/ORBextractor.h:45-111 of the reference) and integration/orbx_slam2_glue.h
(Frame::ComputeStereoMatches, Frame.cc:496-686; ORBmatcher::SearchByBoW, ORBmatcher.cc:182-319)
built by g++ into tests/native/facade_test.cpp, with the cv:: types from the stand-in headers of
tests/native/cv_standin (no OpenCV in this image: the stand-in keeps OpenCV's member names and
semantics, so this proves the facade's marshalling, not OpenCV itself).

* CPU: the program compiles with -Wall -Wextra, and the ORBextractor constructor on a host
  without a GPU throws std::runtime_error naming the failing call (no silent fallback).
* GPU: Frame's two ExtractORB threads (Frame.cc:89-92) on the KITTI fixture pair, the left image
  behind a padded row stride, the stereo glue and SearchByBoW: keypoints, descriptors, uRight and
  depth equal the committed golden digests (tests/golden/fixtures.json), the matches equal the
  restated matcher's.  mvImagePyramid after operator() equals the oracle's levels bytewise, and
  the reference's stereo body (Frame.cc:496-686) run over it equals the glue's device match.
"""
import hashlib
import json
import pathlib
import subprocess

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
GOLDEN = json.loads((ROOT / "tests" / "golden" / "fixtures.json").read_text())


@pytest.fixture(scope="module")
def facade_bin(orbx_lib):
    from my_orb_slam2_amd import build as b
    return b.build_facade_test()


def test_facade_fails_loudly_without_gpu(facade_bin):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    r = subprocess.run([str(facade_bin), "nogpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "orbx_extractor_create" in r.stdout


def _sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,mode", [(0, "threads"), (1, "threads"), (0, "frame"), (1, "frame")])
def test_facade_dropin_sequence(facade_bin, oracle_mod, gpu, tmp_path, seed, mode):
    """threads: Frame's two ExtractORB threads + ComputeStereoMatches; frame: the same Frame
    through orbx_glue::ExtractStereo's single two-image submission (orbx_stereo_frame_view)."""
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
    (tmp_path / "params.txt").write_text(f"{W} {H} {g['params'][0]} {g['mbf']!r}\n")
    r = subprocess.run([str(facade_bin), "run", str(tmp_path)] + (["frame"] if mode == "frame" else []),
                       capture_output=True, text=True, timeout=120)
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
    if mode == "threads":
        # mvImagePyramid straight after operator() (ORBextractor.h:85; refilled at
        # ORBextractor.cc:1129-1154): every level of both views bytewise against the oracle's;
        # the program also checked that Frame.cc:496-686 over these cv::Mat levels gives the
        # glue's uRight / depth (nvalid_ref == nvalid)
        from oracle import OracleExtractor
        for view, img in (("left", L), ("right", R)):
            ox = OracleExtractor(g["params"][0])
            ox(img)
            want = b"".join(ox.level(l).tobytes() for l in range(8))
            got = rd(f"pyr_{view}.bin")
            assert len(got) == len(want), view
            assert got == want, f"mvImagePyramid of the {view} view differs from the oracle's levels"
        assert int(np.frombuffer(rd("nvalid_ref.bin"), np.int32)[0]) == g["n_valid"]


@pytest.mark.gpu
def test_facade_bench_matches_cabi_bench(facade_bin, orbx_lib, gpu, tmp_path):
    """bench.py --workload dropin's loops on the same pairs, 3 tracking sessions each: through
    the facade (facade_test `bench`: a Frame per frame, two ExtractORB threads, the stereo
    glue), through its one-call form (`bench ... frame`: orbx_glue::ExtractStereo) and through
    the bare C ABI (boundary_test `bench`): every session's output digest equal across all
    three (neither the facade nor the two-image submission changes a result)."""
    from my_orb_slam2_amd import build as b
    from my_orb_slam2_amd import synth
    mbf, fx = 386.1448, 718.856
    mb = float(np.float32(mbf) / np.float32(fx))
    for i in range(2):
        L, R = synth.stereo_pair(760 + i, 1241, 376)
        L.tofile(tmp_path / f"pair_{i}_left.raw")
        R.tofile(tmp_path / f"pair_{i}_right.raw")
    (tmp_path / "params.txt").write_text(f"1241 376 2000 {mbf!r} {mb!r} 2\n")
    out = {}
    for name, binp, extra in (("facade", facade_bin, []), ("frame", facade_bin, ["frame"]),
                              ("cabi", b.build_boundary_test(), [])):
        r = subprocess.run([str(binp), "bench", str(tmp_path), "5", "2", "3"] + extra,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, name + ": " + r.stderr
        out[name] = json.loads(r.stdout.strip().splitlines()[-1])
        assert out[name]["trackers"] == 3 and len(out[name]["latency_ms"]) == 15
    assert len(set(out["facade"]["digests"])) == 1, out["facade"]["digests"]
    assert out["facade"]["digests"] == out["cabi"]["digests"] == out["frame"]["digests"]
    assert out["facade"]["mean_stereo_matches"] == out["cabi"]["mean_stereo_matches"] > 0
