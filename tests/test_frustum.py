"""Frame::isInFrustum + MapPoint::PredictScale (src/Frame.cc:285-349, MapPoint.cc:430-444) and
the SearchByProjection window built from them (ORBmatcher.cc:55-80): the projection half of
Tracking::SearchLocalPoints (Tracking.cc:1297-1347).

CPU: the C++ restatement (oracle/orb_frame_oracle.cpp) against a second, numpy restatement of
the same statements; the synthetic local map exercises every rejection.  GPU: k_frustum
(orbx_is_in_frustum / _batch_device) bit for bit against the C++ restatement, one frame and the
256-frame EuRoC batch bench.py --workload euroc times."""
import ctypes
import math

import numpy as np
import pytest

from my_orb_slam2_amd import synth
from my_orb_slam2_amd._lib import KEYPOINT_DTYPE
from my_orb_slam2_amd.features import MAP_POINT_DTYPE, PROJ_QUERY_DTYPE, frame_pose

_libm = ctypes.CDLL("libm.so.6")
_libm.logf.restype = ctypes.c_float
_libm.logf.argtypes = [ctypes.c_float]
_libm.ceilf.restype = ctypes.c_float
_libm.ceilf.argtypes = [ctypes.c_float]
f32 = np.float32


def _keys(seed, n=800, w=752, h=480):
    rng = np.random.default_rng(seed)
    k = np.zeros(n, KEYPOINT_DTYPE)
    k["x"] = rng.uniform(20, w - 20, n)
    k["y"] = rng.uniform(20, h - 20, n)
    k["octave"] = rng.integers(0, 8, n)
    return k, rng.integers(0, 256, (n, 32), dtype=np.uint8)


def _scene(seed, n=2000):
    K4, _ = synth.EUROC_CAM
    bounds = (0.0, 752.0, 0.0, 480.0)
    keys, desc = _keys(seed)
    return synth.local_map_points(seed, keys, desc, n, K4, bounds, mbf=40.0)


def numpy_is_in_frustum(F, mps, skip, cos_lim=0.5, th=1.0):
    """Second restatement, statement by statement in numpy float32 / Python double."""
    q = np.zeros(len(mps), PROJ_QUERY_DTYPE)
    q["radius"] = -1.0
    q["min_level"] = q["max_level"] = q["pred_level"] = -1
    R, t, Ow = F["Rcw"].reshape(3, 3), F["tcw"], F["Ow"]
    n_vis = 0
    for i, m in enumerate(mps):
        if skip is not None and skip[i]:
            continue
        P = m["pos"]
        Pc = []
        for r in range(3):
            s = f32(f32(R[r, 0] * P[0]) + f32(R[r, 1] * P[1]))
            s = f32(s + f32(R[r, 2] * P[2]))
            Pc.append(f32(float(s) + float(t[r])))
        if Pc[2] < f32(0):
            continue
        with np.errstate(divide="ignore", invalid="ignore"):
            invz = f32(f32(1.0) / Pc[2])
            u = f32(f32(f32(F["fx"] * Pc[0]) * invz) + F["cx"])
            v = f32(f32(f32(F["fy"] * Pc[1]) * invz) + F["cy"])
        if u < F["min_x"] or u > F["max_x"] or v < F["min_y"] or v > F["max_y"]:
            continue
        maxd, mind = f32(f32(1.2) * m["max_dist"]), f32(f32(0.8) * m["min_dist"])
        PO = [f32(P[k] - Ow[k]) for k in range(3)]
        ss = 0.0
        for k in range(3):
            ss += float(PO[k]) * float(PO[k])
        dist = f32(math.sqrt(ss))
        if dist < mind or dist > maxd:
            continue
        dot = 0.0
        for k in range(3):
            dot += float(PO[k]) * float(m["normal"][k])
        vc = f32(dot / float(dist))
        if vc < f32(cos_lim):
            continue
        ratio = f32(m["max_dist"] / dist)
        qf = _libm.ceilf(f32(f32(_libm.logf(ratio)) / F["log_scale_factor"]))
        lvl = int(qf) if -2.0 ** 31 <= qf < 2.0 ** 31 else -2 ** 31
        lvl = 0 if lvl < 0 else min(lvl, int(F["nlevels"]) - 1)
        r = f32(2.5) if float(vc) > 0.998 else f32(4.0)
        if th != 1.0:
            r = f32(r * f32(th))
        q[i] = (u, v, f32(u - f32(F["mbf"] * invz)), f32(r * F["scale"][lvl]), lvl - 1, lvl, lvl, 0)
        n_vis += 1
    return q, n_vis


def test_log_scale_factor_is_glibc_logf():
    F = frame_pose(np.eye(3), np.zeros(3), (1, 1, 0, 0), (0, 1, 0, 1), np.ones(8))
    assert F["log_scale_factor"] == _libm.logf(f32(1.2))


@pytest.mark.parametrize("seed", [3, 11])
def test_oracle_matches_numpy_restatement(oracle_mod, seed):
    from oracle import matcher as om
    F, mps, _, skip = _scene(seed, 600)
    qo, no = om.is_in_frustum(F, mps, skip)
    qn, nn = numpy_is_in_frustum(F, mps, skip)
    assert no == nn
    assert qo.tobytes() == qn.tobytes()
    # every kind of outcome occurs: both radii, several levels, rejections and skips
    qv = qo.view(PROJ_QUERY_DTYPE)
    vis = qv["radius"] > 0
    assert 0.55 < vis.mean() < 0.95
    assert len(set(qv["pred_level"][vis].tolist())) >= 6
    r0 = qv["radius"][vis] / F["scale"][qv["pred_level"][vis]]
    assert set(np.round(r0, 3).tolist()) == {2.5, 4.0}
    # th != 1 scales the radius (RGB-D th = 3, Tracking.cc:1340-1343)
    q3, _ = om.is_in_frustum(F, mps, skip, 0.5, 3.0)
    qn3, _ = numpy_is_in_frustum(F, mps, skip, 0.5, 3.0)
    assert q3.tobytes() == qn3.tobytes()


def test_inliers_predict_their_level(oracle_mod):
    """The synthetic map's MapPoints that observe a feature project onto it at the level the
    generator asked for (PredictScale inverts mfMaxDistance = dist * 1.2^(level - 1/2))."""
    from oracle import matcher as om
    K4, _ = synth.EUROC_CAM
    keys, desc = _keys(5)
    F, mps, _, skip = synth.local_map_points(5, keys, desc, 500, K4, (0.0, 752.0, 0.0, 480.0),
                                             inlier_frac=1.0, outside_frac=0.0, skip_frac=0.0)
    q, n = om.is_in_frustum(F, mps, None)
    qv = q.view(PROJ_QUERY_DTYPE)
    assert n >= 0.97 * len(mps)
    vis = qv["radius"] > 0
    # every projection lands near some feature
    d = np.hypot(qv["u"][vis, None] - keys["x"][None, :], qv["v"][vis, None] - keys["y"][None, :])
    assert np.median(d.min(1)) < 1.5


def test_skip_and_empty(oracle_mod):
    from oracle import matcher as om
    F, mps, _, _ = _scene(7, 50)
    q, n = om.is_in_frustum(F, mps, np.ones(len(mps), np.uint8))
    assert n == 0 and (q.view(PROJ_QUERY_DTYPE)["radius"] == -1).all()
    q, n = om.is_in_frustum(F, mps[:0], None)
    assert n == 0 and len(q) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [3, 11, 29])
def test_gpu_frustum_one_frame(oracle_mod, orbx_lib, gpu, seed):
    from oracle import matcher as om
    from my_orb_slam2_amd.features import is_in_frustum
    F, mps, _, skip = _scene(seed, 3000)
    qg, ng = is_in_frustum(F, mps, skip)
    qo, no = om.is_in_frustum(F, mps, skip)
    assert ng == no
    bad = np.nonzero(qg.view(np.uint8).reshape(-1, 32) != qo.reshape(-1, 32))[0]
    assert bad.size == 0, f"queries differ at MapPoints {np.unique(bad)[:8]}"
    q3, _ = is_in_frustum(F, mps, skip, 0.5, 3.0)
    qo3, _ = om.is_in_frustum(F, mps, skip, 0.5, 3.0)
    assert q3.tobytes() == qo3.tobytes()
    qe, ne = is_in_frustum(F, mps[:0])
    assert ne == 0 and len(qe) == 0
