"""Frame geometry around the matchers: undistortion (cvUndistortPoints, OpenCV 3.2 restated),
image bounds and the feature grid.  CPU: the restatement against a numpy float64 reading and
the host bounds; GPU: device undistortion and grid against the restatement."""
import numpy as np
import pytest

from my_orb_slam2_amd import synth
from my_orb_slam2_amd._lib import KEYPOINT_DTYPE
from my_orb_slam2_amd.features import assign_features_to_grid, image_bounds

CAMS = {"euroc": synth.EUROC_CAM, "tum1": synth.TUM1_CAM,
        "rational": ((500.0, 501.0, 320.5, 240.25), (0.1, -0.05, 0.001, -0.002, 0.01, 0.02, -0.01, 0.005))}


def undistort_np(xy, K4, dist):
    """cvUndistortPoints (OpenCV 3.2) in numpy float64, same operation order."""
    k = np.zeros(8)
    d = np.asarray(dist, np.float32).astype(np.float64)
    k[:len(d)] = d
    fx, fy, cx, cy = (float(np.float32(v)) for v in K4)
    ifx, ify = 1.0 / fx, 1.0 / fy
    x = (xy[:, 0].astype(np.float64) - cx) * ifx
    y = (xy[:, 1].astype(np.float64) - cy) * ify
    x0, y0 = x.copy(), y.copy()
    for _ in range(5):
        r2 = x * x + y * y
        icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
        dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x)
        dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y
        x = (x0 - dx) * icdist
        y = (y0 - dy) * icdist
    xx = fx * x + 0.0 * y + cx
    yy = 0.0 * x + fy * y + cy
    ww = 1.0 / (0.0 * x + 0.0 * y + 1.0)
    return np.stack([(xx * ww).astype(np.float32), (yy * ww).astype(np.float32)], 1)


def _keys(n, w=752, h=480, seed=0):
    rng = np.random.default_rng(seed)
    k = np.zeros(n, KEYPOINT_DTYPE)
    k["x"] = rng.uniform(0, w, n)
    k["y"] = rng.uniform(0, h, n)
    k["octave"] = rng.integers(0, 8, n)
    k["angle"] = rng.uniform(0, 360, n)
    return k


@pytest.mark.parametrize("cam", list(CAMS))
def test_undistort_oracle_vs_numpy(cam):
    from oracle import matcher as om
    K4, dist = CAMS[cam]
    k = _keys(3000)
    got = om.undistort_keypoints(k, K4, dist)
    want = undistort_np(np.stack([k["x"], k["y"]], 1).astype(np.float32), K4, dist)
    np.testing.assert_array_equal(got.view(np.int32), want.view(np.int32))


def test_undistort_zero_k1_copies():
    from oracle import matcher as om
    k = _keys(50)
    got = om.undistort_keypoints(k, synth.EUROC_CAM[0], (0.0, 0.1, 0.01, 0.01))
    np.testing.assert_array_equal(got[:, 0], k["x"])


@pytest.mark.parametrize("cam", list(CAMS))
def test_image_bounds_host(orbx_lib, cam):
    from oracle import matcher as om
    K4, dist = CAMS[cam]
    assert image_bounds(K4, dist, 752, 480) == om.image_bounds(K4, dist, 752, 480)
    assert image_bounds(K4, (0, 0, 0, 0), 640, 480) == (0.0, 640.0, 0.0, 480.0)


@pytest.mark.gpu
@pytest.mark.parametrize("cam", list(CAMS))
def test_undistort_gpu(oracle_mod, orbx_lib, gpu, cam):
    from oracle import matcher as om
    from my_orb_slam2_amd.features import undistort_keypoints
    K4, dist = CAMS[cam]
    k = _keys(5000, seed=3)
    un = undistort_keypoints(k, K4, dist)
    want = om.undistort_keypoints(k, K4, dist)
    np.testing.assert_array_equal(un["x"].view(np.int32), want[:, 0].view(np.int32))
    np.testing.assert_array_equal(un["y"].view(np.int32), want[:, 1].view(np.int32))
    np.testing.assert_array_equal(un["octave"], k["octave"])


@pytest.mark.gpu
def test_grid_gpu(orbx_lib, gpu):
    import torch
    from my_orb_slam2_amd.features import assign_grid_device
    for seed, n in [(0, 2000), (1, 1), (2, 0), (3, 4500)]:
        k = _keys(n, seed=seed)
        if n >= 5:
            k["x"][:5] = [0.0, 751.99, -3.0, 5.875, 760.0]   # borders and outside
        bmin_x, bmax_x, bmin_y, bmax_y = image_bounds(*synth.EUROC_CAM, 752, 480)
        g = assign_features_to_grid(k, bmin_x, bmax_x, bmin_y, bmax_y)
        dk = torch.from_numpy(k.view(np.uint8).copy()).to(gpu) if n else torch.zeros(28, dtype=torch.uint8, device=gpu)
        off = torch.zeros(64 * 48 + 1, dtype=torch.int32, device=gpu)
        feat = torch.full((max(n, 1),), -1, dtype=torch.int32, device=gpu)
        assign_grid_device(dk, n, bmin_x, bmax_x, bmin_y, bmax_y, off, feat)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(off.cpu().numpy(), g.off)
        np.testing.assert_array_equal(feat.cpu().numpy()[:len(g.feat)], g.feat)


@pytest.mark.gpu
def test_grid_and_undistort_batch_gpu(oracle_mod, orbx_lib, gpu):
    """Batched undistortion + grid over frames laid out like orbx_batch_view (padded slots
    with garbage, one empty frame, one dense frame with crowded cells)."""
    import torch
    from oracle import matcher as om
    from my_orb_slam2_amd.features import (assign_grid_batch_device,
                                           undistort_keypoints_batch_device)
    K4, dist = synth.EUROC_CAM
    stride, ns = 1500, [1000, 0, 1500, 37, 1200]
    frames = []
    allk = np.zeros(len(ns) * stride, KEYPOINT_DTYPE)
    allk["x"] = 1e30   # padding garbage
    for f, n in enumerate(ns):
        k = _keys(n, seed=10 + f)
        if f == 2:   # crowd one corner so cells hold many features
            k["x"][:400] = np.random.default_rng(0).uniform(100, 112, 400)
            k["y"][:400] = np.random.default_rng(1).uniform(200, 211, 400)
        allk[f * stride:f * stride + n] = k
        frames.append(k)
    dk = torch.from_numpy(allk.view(np.uint8).copy()).to(gpu)
    dn = torch.tensor(ns, dtype=torch.int32, device=gpu)
    dun = torch.zeros_like(dk)
    undistort_keypoints_batch_device(K4, dist, dk, stride, dn, len(ns), dun)
    bounds = image_bounds(K4, dist, 752, 480)
    off = torch.full((len(ns), 64 * 48 + 1), -7, dtype=torch.int32, device=gpu)
    feat = torch.full((len(ns), stride), -7, dtype=torch.int32, device=gpu)
    assign_grid_batch_device(dun, stride, dn, len(ns), bounds, off, feat)
    torch.cuda.synchronize()
    un = dun.cpu().numpy().view(KEYPOINT_DTYPE)
    off, feat = off.cpu().numpy(), feat.cpu().numpy()
    for f, (n, k) in enumerate(zip(ns, frames)):
        want = om.undistort_keypoints(k, K4, dist) if n else np.zeros((0, 2), np.float32)
        got = un[f * stride:f * stride + n]
        np.testing.assert_array_equal(got["x"].view(np.int32), want[:, 0].view(np.int32))
        np.testing.assert_array_equal(got["y"].view(np.int32), want[:, 1].view(np.int32))
        ku = k.copy()
        ku["x"], ku["y"] = want[:, 0], want[:, 1]
        g = assign_features_to_grid(ku, *bounds)
        np.testing.assert_array_equal(off[f], g.off)
        np.testing.assert_array_equal(feat[f, :len(g.feat)], g.feat)


@pytest.mark.parametrize("rgb,c", [(0, 3), (1, 3), (0, 4), (1, 4)])
def test_cvt_gray_oracle_vs_numpy(rgb, c):
    from oracle import matcher as om
    img = np.random.default_rng(c + rgb).integers(0, 256, (37, 53, c), dtype=np.uint8)
    r, g, b = (img[..., 0], img[..., 1], img[..., 2]) if rgb else (img[..., 2], img[..., 1], img[..., 0])
    r, g, b = (v.astype(np.int64) for v in (r, g, b))
    want = ((r * 4899 + g * 9617 + b * 1868 + 8192) >> 14).astype(np.uint8)
    np.testing.assert_array_equal(om.cvt_gray(img, rgb), want)


@pytest.mark.gpu
@pytest.mark.parametrize("rgb,c", [(0, 3), (1, 3), (0, 4), (1, 4)])
def test_cvt_gray_gpu(orbx_lib, gpu, rgb, c):
    from oracle import matcher as om
    from my_orb_slam2_amd.features import cvt_color_gray
    img = np.random.default_rng(7).integers(0, 256, (376, 1241, c), dtype=np.uint8)
    np.testing.assert_array_equal(cvt_color_gray(img, bool(rgb)), om.cvt_gray(img, rgb))
