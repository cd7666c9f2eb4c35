"""Committed golden fixtures (tests/golden/make_golden.py): the CPU restatement must keep
reproducing them, and the HIP path must reproduce them on the GPU."""
import hashlib
import json
import pathlib

import numpy as np
import pytest

from my_orb_slam2_amd import synth

GOLD = pathlib.Path(__file__).resolve().parent / "golden"
FIX = json.loads((GOLD / "fixtures.json").read_text())
MBF = 386.1448


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _input(spec):
    if spec[0] == "frame":
        return synth.frame(spec[1], spec[2], spec[3])
    if spec[0] == "stereo_pair":
        return synth.stereo_pair(spec[1], spec[2], spec[3])
    return synth.edge_cases()[spec[1]]


def _run(make, name):
    case = FIX[name]
    inp = _input(case["input"])
    if case["input"][0] == "stereo_pair":
        assert [sha(inp[0]), sha(inp[1])] == case["input_sha256"], "synthetic input changed"
    else:
        assert sha(inp) == case["input_sha256"], "synthetic input changed"
    return case, inp


def _check_small(ext):
    case, img = _run(None, "small_320x240_seed42")
    k, d = ext(img)
    ref = np.load(GOLD / "small_320x240_seed42.npz")
    assert k.tobytes() == ref["keypoints"].tobytes()
    assert np.array_equal(d, ref["descriptors"])


def _check_stereo(make, stereo, seed):
    case, (L, R) = _run(None, f"kitti_stereo_seed{seed}")
    l, r = make(*case["params"]), make(*case["params"])
    kl, dl = l(L)
    kr, dr = r(R)
    u, dep, nv = stereo(l, r, len(kl), case["mbf"], case["mb"])
    h = case["sha256"]
    assert sha(kl) == h["kps_left"] and sha(dl) == h["desc_left"]
    assert sha(kr) == h["kps_right"] and sha(dr) == h["desc_right"]
    assert sha(u) == h["uRight"] and sha(dep) == h["depth"] and nv == case["n_valid"]


def _check_edges(make):
    for name in ("zeros", "white", "checker8", "tiny64"):
        case, img = _run(None, f"edge_{name}")
        k, d = make(*case["params"])(img)
        assert len(k) == case["n"]
        assert sha(k) == case["sha256"]["kps"]
        assert (d is None) == (case["sha256"]["desc"] is None)
        if d is not None:
            assert sha(d) == case["sha256"]["desc"]


# ---- CPU restatement ----
def test_oracle_small(oracle_mod):
    _check_small(oracle_mod.OracleExtractor(500, 1.2, 8, 20, 7))


@pytest.mark.parametrize("seed", [0, 1])
def test_oracle_kitti_stereo(oracle_mod, seed):
    _check_stereo(lambda *p: oracle_mod.OracleExtractor(*p),
                  lambda l, r, n, mbf, mb: oracle_mod.stereo_match(l, r, n, mbf, mb), seed)


def test_oracle_edges(oracle_mod):
    _check_edges(lambda *p: oracle_mod.OracleExtractor(*p))


# ---- HIP path ----
@pytest.mark.gpu
def test_gpu_small(orbx_lib, gpu):
    import my_orb_slam2_amd as m
    _check_small(m.ORBextractor(500, 1.2, 8, 20, 7))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1])
def test_gpu_kitti_stereo(orbx_lib, gpu, seed):
    import my_orb_slam2_amd as m
    _check_stereo(lambda *p: m.ORBextractor(*p),
                  lambda l, r, n, mbf, mb: m.compute_stereo_matches(l, r, mbf, mb), seed)


@pytest.mark.gpu
def test_gpu_edges(orbx_lib, gpu):
    import my_orb_slam2_amd as m
    _check_edges(lambda *p: m.ORBextractor(*p))
