"""Seeded synthetic grayscale frames (harness data, not part of the hot path).

There are no datasets in the build image (no KITTI/TUM/EuRoC), so tests and bench.py use
frames generated here, as SURVEY.md §8(d) prescribes: piecewise-constant random rectangles
and disks (intensities U[0,255]) over a low-frequency gradient, plus Gaussian noise, clipped
to uint8.  Stereo pairs are rendered from one layered scene: every shape carries a
disparity d in [2, 64] px and the right view draws it shifted left by d (rectified,
row-aligned), nearer shapes painted last; the two views get independent noise.
"""
from __future__ import annotations

import numpy as np

KITTI = dict(width=1241, height=376, nfeatures=2000, fx=718.856, mbf=386.1448)  # KITTI00-02.yaml
TUM = dict(width=640, height=480, nfeatures=1000)                             # TUM1.yaml
EUROC = dict(width=752, height=480, nfeatures=1000)                           # EuRoC.yaml
# camera intrinsics (fx, fy, cx, cy) and distortion (k1, k2, p1, p2[, k3]) of the examples
EUROC_CAM = ((458.654, 457.296, 367.215, 248.375),
             (-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05))   # Monocular/EuRoC.yaml:8-16
TUM1_CAM = ((517.306408, 516.469215, 318.643040, 255.313989),
            (0.262383, -0.953104, -0.005358, 0.002628, 1.163314))     # Monocular/TUM1.yaml:8-17


def _scene(rng, width, height, n_rect, n_disk):
    shapes = []
    for _ in range(n_rect):
        w = int(rng.integers(6, max(7, width // 6)))
        h = int(rng.integers(6, max(7, height // 5)))
        x0 = int(rng.integers(-w // 2, width))
        y0 = int(rng.integers(-h // 2, height))
        shapes.append(("rect", x0, y0, w, h, float(rng.uniform(0, 255)), float(rng.uniform(2, 64))))
    for _ in range(n_disk):
        r = float(rng.uniform(3, max(4, min(width, height) / 10)))
        cx = float(rng.uniform(0, width))
        cy = float(rng.uniform(0, height))
        shapes.append(("disk", cx, cy, r, 0, float(rng.uniform(0, 255)), float(rng.uniform(2, 64))))
    shapes.sort(key=lambda s: s[6])  # far (small disparity) first
    gx, gy, g0 = rng.uniform(-60, 60), rng.uniform(-60, 60), rng.uniform(60, 190)
    return shapes, (gx, gy, g0)


def _render(shapes, grad, width, height, shift_scale):
    gx, gy, g0 = grad
    yy, xx = np.mgrid[0:height, 0:width].astype(np.float32)
    img = g0 + gx * (xx / width - 0.5) + gy * (yy / height - 0.5)
    for kind, a, b, c, d, val, disp in shapes:
        dx = -disp * shift_scale
        if kind == "rect":
            x0 = int(round(a + dx))
            x1, y0, y1 = x0 + c, b, b + d
            x0c, x1c = max(0, x0), min(width, x1)
            y0c, y1c = max(0, y0), min(height, y1)
            if x0c < x1c and y0c < y1c:
                img[y0c:y1c, x0c:x1c] = val
        else:
            cx, cy, r = a + dx, b, c
            xa, xb = max(0, int(cx - r) - 1), min(width, int(cx + r) + 2)
            ya, yb = max(0, int(cy - r) - 1), min(height, int(cy + r) + 2)
            if xa < xb and ya < yb:
                sub = (xx[ya:yb, xa:xb] - cx) ** 2 + (yy[ya:yb, xa:xb] - cy) ** 2 <= r * r
                img[ya:yb, xa:xb][sub] = val
    return img


def frame(seed: int, width: int = 1241, height: int = 376, n_rect: int | None = None,
          n_disk: int | None = None, noise: float = 3.0) -> np.ndarray:
    """One monocular uint8 frame (H x W), deterministic in `seed`."""
    rng = np.random.default_rng(seed)
    area = width * height
    n_rect = n_rect if n_rect is not None else max(8, area // 2500)
    n_disk = n_disk if n_disk is not None else max(4, area // 4000)
    shapes, grad = _scene(rng, width, height, n_rect, n_disk)
    img = _render(shapes, grad, width, height, 0.0)
    img += rng.normal(0.0, noise, size=img.shape).astype(np.float32)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def stereo_pair(seed: int, width: int = 1241, height: int = 376, noise_l: float = 3.0,
                noise_r: float = 2.0):
    """A rectified (left, right) uint8 pair rendered from one layered scene."""
    rng = np.random.default_rng(seed)
    area = width * height
    shapes, grad = _scene(rng, width, height, max(8, area // 2500), max(4, area // 4000))
    left = _render(shapes, grad, width, height, 0.0)
    right = _render(shapes, grad, width, height, 1.0)
    left += rng.normal(0.0, noise_l, size=left.shape).astype(np.float32)
    right += rng.normal(0.0, noise_r, size=right.shape).astype(np.float32)
    to8 = lambda a: np.clip(np.rint(a), 0, 255).astype(np.uint8)
    return to8(left), to8(right)


def edge_cases(width: int = 640, height: int = 480):
    """Named edge-case frames: blank, saturated, checkerboard (score ties), tiny."""
    yy, xx = np.mgrid[0:height, 0:width]
    return {
        "zeros": np.zeros((height, width), np.uint8),
        "white": np.full((height, width), 255, np.uint8),
        "checker8": (((xx // 8 + yy // 8) % 2) * 255).astype(np.uint8),
        "tiny64": frame(7, 64, 64),
    }


# ---- matcher workloads ----------------------------------------------------------------------

def scale_tables(nlevels: int = 8, scale_factor: float = 1.2):
    """mvScaleFactors / mvLevelSigma2 / mvInvLevelSigma2 as ORBextractor builds them
    (src/ORBextractor.cc:415-433: float products of the double scale factor)."""
    s = [np.float32(1.0)]
    for _ in range(1, nlevels):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(scale_factor))))
    s = np.array(s, np.float32)
    s2 = (s * s).astype(np.float32)
    return s, s2, (np.float32(1.0) / s2).astype(np.float32)


def _octaves(rng, n, nlevels=8, scale_factor=1.2):
    w = np.float64(scale_factor) ** -np.arange(nlevels)
    return rng.choice(nlevels, size=n, p=w / w.sum()).astype(np.int32)


def _flip(rng, desc, nflip):
    d = desc.copy()
    for i, k in enumerate(nflip):
        if k:
            bits = rng.choice(256, size=int(k), replace=False)
            np.bitwise_xor.at(d[i], bits // 8, (1 << (bits % 8)).astype(np.uint8))
    return d


def _node_of(desc, nodes):
    # a stand-in vocabulary: the node a descriptor falls into depends on a few of its bits,
    # so near-identical descriptors usually (not always) share it; ids are sparse
    key = (desc[:, 0].astype(np.int64) * 131 + desc[:, 5].astype(np.int64) * 7) % nodes
    return 1000 + 3 * key


def feature_pair(seed: int, n1: int = 1000, n2: int = 1000, width: int = 752,
                 height: int = 480, match_frac: float = 0.6, nodes: int = 40,
                 stereo_frac: float = 0.5, rotation: float = 25.0, dup_frac: float = 0.05,
                 single_node: bool = False, max_flip: int = 40, nlevels: int = 8):
    """Two correlated feature sets (Frame/KeyFrame arrays) for the matcher tests.

    A fraction of set-2 features are noisy copies of set-1 features (position +-2 px, angle
    rotated by `rotation` with 10% outliers, 0..max_flip flipped descriptor bits); a few
    set-2 descriptors are duplicated onto neighbours so distance ties occur.  Returns
    (f1, f2, truth) with truth[i] = the set-2 copy of set-1 feature i or -1.
    """
    from .features import FeatureSet, assign_features_to_grid, feature_vector
    from ._lib import KEYPOINT_DTYPE
    rng = np.random.default_rng(seed)
    k1 = np.zeros(n1, KEYPOINT_DTYPE)
    k1["x"] = rng.uniform(0, width, n1)
    k1["y"] = rng.uniform(0, height, n1)
    k1["octave"] = _octaves(rng, n1, nlevels)
    k1["angle"] = rng.uniform(0, 360, n1)
    k1["size"] = 31
    k1["class_id"] = -1
    d1 = rng.integers(0, 256, (n1, 32), dtype=np.uint8)

    nm = min(int(match_frac * min(n1, n2)), n1, n2)
    src = rng.choice(n1, size=nm, replace=False)
    dst = rng.choice(n2, size=nm, replace=False)
    k2 = np.zeros(n2, KEYPOINT_DTYPE)
    k2["x"] = rng.uniform(0, width, n2)
    k2["y"] = rng.uniform(0, height, n2)
    k2["octave"] = _octaves(rng, n2, nlevels)
    k2["angle"] = rng.uniform(0, 360, n2)
    k2["size"] = 31
    k2["class_id"] = -1
    d2 = rng.integers(0, 256, (n2, 32), dtype=np.uint8)
    k2["x"][dst] = np.clip(k1["x"][src] + rng.normal(0, 2, nm), 0, width - 1e-3)
    k2["y"][dst] = np.clip(k1["y"][src] + rng.normal(0, 2, nm), 0, height - 1e-3)
    k2["octave"][dst] = np.clip(k1["octave"][src] + rng.integers(-1, 2, nm), 0, nlevels - 1)
    ang = (k1["angle"][src] - rotation + rng.normal(0, 4, nm)) % 360
    out = rng.random(nm) < 0.1
    ang[out] = rng.uniform(0, 360, out.sum())
    k2["angle"][dst] = ang.astype(np.float32)
    d2[dst] = _flip(rng, d1[src], rng.integers(0, max_flip + 1, nm))
    # duplicated descriptors next to each other: exact distance ties
    nd = int(dup_frac * n2)
    if nd:
        a = rng.choice(n2, size=nd, replace=False)
        b = rng.choice(n2, size=nd, replace=False)
        d2[b] = d2[a]
        k2["x"][b] = np.clip(k2["x"][a] + rng.uniform(-3, 3, nd), 0, width - 1e-3)
        k2["y"][b] = np.clip(k2["y"][a] + rng.uniform(-3, 3, nd), 0, height - 1e-3)
        k2["octave"][b] = k2["octave"][a]
    truth = np.full(n1, -1, np.int64)
    truth[src] = dst

    def stereo(keys):
        ur = np.full(len(keys), -1.0, np.float32)
        s = rng.random(len(keys)) < stereo_frac
        ur[s] = (keys["x"][s] - rng.uniform(2, 64, s.sum())).astype(np.float32)
        return ur

    def fset(keys, desc):
        nodes_of = np.zeros(len(keys), np.int64) if single_node else _node_of(desc, nodes)
        fs = FeatureSet(keys, desc, stereo(keys), feature_vector(nodes_of),
                        assign_features_to_grid(keys, 0.0, width, 0.0, height))
        return fs

    return fset(k1, d1), fset(k2, d2), truth


def projection_queries(seed: int, f1, f2, truth, th: float = 3.0, nlevels: int = 8,
                       mode_levels: str = "frame", inactive_frac: float = 0.05,
                       max_flip: int = 20):
    """MapPoint projections into f2 built from f1's features (for the projection searches):
    matched features project near their f2 copy, the rest anywhere.  Returns
    (queries PROJ_QUERY_DTYPE, descriptors)."""
    from .features import PROJ_QUERY_DTYPE
    rng = np.random.default_rng(seed)
    scale, _, _ = scale_tables(nlevels)
    n = f1.n
    q = np.zeros(n, PROJ_QUERY_DTYPE)
    has = truth >= 0
    tx = np.where(has, f2.keys["x"][np.maximum(truth, 0)], rng.uniform(0, 752, n))
    ty = np.where(has, f2.keys["y"][np.maximum(truth, 0)], rng.uniform(0, 480, n))
    q["u"] = (tx + rng.normal(0, 1.5, n)).astype(np.float32)
    q["v"] = (ty + rng.normal(0, 1.5, n)).astype(np.float32)
    pred = np.where(has, f2.keys["octave"][np.maximum(truth, 0)], f1.keys["octave"])
    pred = np.clip(pred + rng.integers(-1, 2, n), 0, nlevels - 1).astype(np.int32)
    q["pred_level"] = pred
    q["radius"] = (np.float32(th) * scale[pred]).astype(np.float32)
    if mode_levels == "frame":
        q["min_level"] = pred - 1
        q["max_level"] = pred
    else:
        q["min_level"] = -1
        q["max_level"] = -1
    ur = f2.u_right[np.maximum(truth, 0)] if f2.u_right is not None else np.full(n, -1, np.float32)
    q["ur"] = np.where(has & (ur > 0), ur + rng.normal(0, 1.0, n), q["u"] - 30).astype(np.float32)
    q["angle"] = f1.keys["angle"]
    q["radius"][rng.random(n) < inactive_frac] = -1.0
    desc = _flip(rng, f1.desc, rng.integers(0, max_flip + 1, n))
    return q, desc


def local_map_queries(seed: int, keys_un, desc, n_queries: int, width: int = 752,
                      height: int = 480, th: float = 1.0, inlier_frac: float = 0.6,
                      nlevels: int = 8, max_flip: int = 24):
    """Projected local-map MapPoints for one frame (Tracking::SearchLocalPoints inputs,
    Tracking.cc:1297-1347): `inlier_frac` of the queries are MapPoints observed as one of the
    frame's features (projection within ~1 px of its undistorted position, descriptor with
    0..max_flip flipped bits, predicted level = octave +-1), the rest land anywhere with
    random descriptors.  radius = th * RadiusByViewingCos (2.5 or 4.0, Tracking.cc:1353-1359)
    * scale[pred] as ORBmatcher.cc:75-80 computes it.  Returns (queries, descriptors)."""
    from .features import PROJ_QUERY_DTYPE
    rng = np.random.default_rng(seed)
    scale, _, _ = scale_tables(nlevels)
    n = len(keys_un)
    q = np.zeros(n_queries, PROJ_QUERY_DTYPE)
    nin = min(n, int(round(inlier_frac * n_queries)))
    src = rng.choice(n, nin, replace=False) if nin else np.zeros(0, np.int64)
    u = rng.uniform(0, width, n_queries)
    v = rng.uniform(0, height, n_queries)
    u[:nin] = keys_un["x"][src] + rng.normal(0, 0.7, nin)
    v[:nin] = keys_un["y"][src] + rng.normal(0, 0.7, nin)
    pred = rng.integers(0, nlevels, n_queries)
    pred[:nin] = np.clip(keys_un["octave"][src] + rng.integers(-1, 2, nin), 0, nlevels - 1)
    r = np.where(rng.random(n_queries) < 0.7, np.float32(2.5), np.float32(4.0))
    d = rng.integers(0, 256, (n_queries, 32), dtype=np.uint8)
    d[:nin] = _flip(rng, desc[src], rng.integers(0, max_flip + 1, nin))
    perm = rng.permutation(n_queries)   # MapPoint order is unrelated to feature order
    q["u"], q["v"] = u.astype(np.float32)[perm], v.astype(np.float32)[perm]
    q["ur"] = -1.0
    pred = pred.astype(np.int32)[perm]
    q["pred_level"], q["min_level"], q["max_level"] = pred, pred - 1, pred
    q["radius"] = (np.float32(th) * r[perm] * scale[pred]).astype(np.float32)
    q["angle"] = 0.0
    return q, np.ascontiguousarray(d[perm])


def local_map_points(seed: int, keys_un, desc, n_points: int, K4, bounds, width: int = 752,
                     height: int = 480, th: float = 1.0, inlier_frac: float = 0.6,
                     outside_frac: float = 0.12, nlevels: int = 8, scale_factor: float = 1.2,
                     max_flip: int = 24, skip_frac: float = 0.05, mbf: float = 0.0):
    """A 3-D local map for one frame (Tracking::SearchLocalPoints inputs, Tracking.cc:1297-1347,
    before isInFrustum): a camera pose and `n_points` MapPoints (orbx_map_point records) with
    descriptors.  `inlier_frac` of them are observations of the frame's own features: they
    project within ~1 px of the feature, with a descriptor 0..max_flip bits away and a
    mfMaxDistance that puts PredictScale at the feature's octave +-1; the rest land anywhere in
    the image with random descriptors; `outside_frac` fail one of isInFrustum's tests (behind
    the camera, outside the image bounds, outside the scale-invariance distances, viewing
    angle above 60 degrees).  Normals are the viewing direction turned by up to 40 degrees (a
    tenth of them exactly the viewing direction: RadiusByViewingCos 2.5).  `skip_frac` of the
    MapPoints are flagged as already matched in the frame (mnLastFrameSeen).  Returns
    (frame_pose record, map points, descriptors [n, 32], skip mask)."""
    from .features import MAP_POINT_DTYPE, frame_pose
    rng = np.random.default_rng(seed)
    scale, _, _ = scale_tables(nlevels, scale_factor)
    fx, fy, cx, cy = (float(v) for v in K4)
    Rcw = _rot(rng, 20.0)
    tcw = rng.normal(0, 1.0, 3)
    pose = frame_pose(Rcw, tcw, K4, bounds, scale, mbf=mbf, scale_factor=scale_factor)
    R = Rcw.astype(np.float64)
    n = len(keys_un)
    nin = min(n, int(round(inlier_frac * n_points)))
    src = rng.choice(n, nin, replace=False) if nin else np.zeros(0, np.int64)
    u = rng.uniform(bounds[0] + 1, bounds[1] - 1, n_points)
    v = rng.uniform(bounds[2] + 1, bounds[3] - 1, n_points)
    u[:nin] = keys_un["x"][src] + rng.normal(0, 0.7, nin)
    v[:nin] = keys_un["y"][src] + rng.normal(0, 0.7, nin)
    lvl = rng.integers(0, nlevels, n_points)
    lvl[:nin] = np.clip(keys_un["octave"][src] + rng.integers(-1, 2, nin), 0, nlevels - 1)
    Z = rng.uniform(2.0, 30.0, n_points)
    Pc = np.stack([(u - cx) / fx * Z, (v - cy) / fy * Z, Z], 1)
    P = (Pc - tcw[None, :]) @ R                      # Rcw^T (Pc - tcw), row vectors
    Ow = -(R.T @ tcw)
    PO = P - Ow[None, :]
    dist = np.linalg.norm(PO, axis=1)
    # PredictScale = ceil(log(maxD / dist) / log(1.2)) = lvl: maxD = dist * 1.2^(lvl - 0.5)
    maxd = dist * float(scale_factor) ** (lvl - 0.5)
    mind = maxd / float(scale[nlevels - 1])
    # normals: the viewing direction turned by up to 40 degrees
    dirn = PO / dist[:, None]
    nrm = np.empty_like(dirn)
    for i in range(n_points):
        nrm[i] = _rot(rng, 40.0) @ dirn[i] if rng.random() > 0.1 else dirn[i]
    # failures of isInFrustum's tests
    kind = np.where(rng.random(n_points) < outside_frac, rng.integers(0, 5, n_points), -1)
    kind[:nin] = -1
    beh = kind == 0                                    # behind the camera
    P[beh] = ((Pc[beh] * np.array([1, 1, -1.0])) - tcw) @ R
    side = kind == 1                                   # outside the image bounds
    P[side] = ((np.stack([(u[side] - cx + width) / fx * Z[side], Pc[side, 1], Z[side]], 1))
               - tcw) @ R
    far = kind == 2                                    # beyond 1.2 * mfMaxDistance
    maxd[far] = dist[far] / 1.5
    near = kind == 3                                   # below 0.8 * mfMinDistance
    mind[near] = dist[near] * 1.5
    maxd[near] = np.maximum(maxd[near], mind[near] * 2)
    ang = kind == 4                                    # viewing angle above 60 degrees
    for i in np.nonzero(ang)[0]:
        ax = np.cross(dirn[i], rng.normal(size=3))
        ax /= np.linalg.norm(ax)
        a = np.deg2rad(rng.uniform(65, 120))
        nrm[i] = dirn[i] * np.cos(a) + np.cross(ax, dirn[i]) * np.sin(a)
    mp = np.zeros(n_points, MAP_POINT_DTYPE)
    mp["pos"] = P.astype(np.float32)
    mp["normal"] = nrm.astype(np.float32)
    mp["max_dist"] = maxd.astype(np.float32)
    mp["min_dist"] = mind.astype(np.float32)
    d = rng.integers(0, 256, (n_points, 32), dtype=np.uint8)
    d[:nin] = _flip(rng, desc[src], rng.integers(0, max_flip + 1, nin))
    skip = (rng.random(n_points) < skip_frac).astype(np.uint8)
    perm = rng.permutation(n_points)   # MapPoint order is unrelated to feature order
    return pose, mp[perm], np.ascontiguousarray(d[perm]), skip[perm]


def _rot(rng, max_deg):
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    a = np.deg2rad(rng.uniform(-max_deg, max_deg))
    Kx = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    return np.eye(3) + np.sin(a) * Kx + (1 - np.cos(a)) * Kx @ Kx


def keyframe_pair(seed: int, n1: int = 1000, n2: int = 1000, width: int = 752,
                  height: int = 480, fx: float = 458.654, fy: float = 457.296,
                  cx: float = 367.215, cy: float = 248.375, baseline: float = 0.5,
                  match_frac: float = 0.6, nodes: int = 40, single_node: bool = False,
                  stereo_frac: float = 0.3):
    """Two keyframes observing one random 3D scene (LocalMapping's SearchForTriangulation
    workload): set-2 copies of set-1 features sit at the true projection (+-0.5 px), so the
    epipolar test passes for them.  Returns (kf1, kf2, F12 float32 3x3, (ex, ey), truth).
    F12 = K^-T [t12]x R12 K^-1 as LocalMapping::ComputeF12 (LocalMapping.cc:612-629); the
    epipole with the float expressions of ORBmatcher.cc:712-715."""
    f1, f2, truth = feature_pair(seed, n1, n2, width, height, match_frac, nodes, stereo_frac,
                                 rotation=5.0, single_node=single_node)
    from .features import assign_features_to_grid
    rng = np.random.default_rng(seed + 7919)
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1.0]])
    R1w, t1w = np.eye(3), np.zeros(3)
    R2w = _rot(rng, 5.0)
    # baseline direction: sideways and/or forward, so the epipole is sometimes in view
    C2w = baseline * np.array([rng.uniform(-1, 1), rng.uniform(-0.2, 0.2), rng.uniform(-1.2, 1.2)])
    t2w = -R2w @ C2w
    src = np.nonzero(truth >= 0)[0]
    dst = truth[src]
    z = rng.uniform(2.0, 25.0, len(src))
    P = np.stack([(f1.keys["x"][src] - cx) / fx * z, (f1.keys["y"][src] - cy) / fy * z, z], 1)
    Pc2 = P @ R2w.T + t2w
    u2 = fx * Pc2[:, 0] / Pc2[:, 2] + cx + rng.normal(0, 0.5, len(src))
    v2 = fy * Pc2[:, 1] / Pc2[:, 2] + cy + rng.normal(0, 0.5, len(src))
    f2.keys["x"][dst] = np.clip(u2, 0, width - 1e-3)
    f2.keys["y"][dst] = np.clip(v2, 0, height - 1e-3)
    f2.grid = assign_features_to_grid(f2.keys, 0.0, width, 0.0, height)
    R12 = R1w @ R2w.T
    t12 = -R1w @ R2w.T @ t2w + t1w
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
    Kinv = np.linalg.inv(K)
    F12 = (Kinv.T @ tx @ R12 @ Kinv).astype(np.float32)
    Cw = (-R1w.T @ t1w).astype(np.float32)
    C2 = (R2w.astype(np.float32) @ Cw + t2w.astype(np.float32)).astype(np.float32)
    invz = np.float32(1.0) / C2[2]
    ex = np.float32(np.float32(np.float32(fx) * C2[0]) * invz) + np.float32(cx)
    ey = np.float32(np.float32(np.float32(fy) * C2[1]) * invz) + np.float32(cy)
    return f1, f2, F12, (float(ex), float(ey)), truth


def write_vocabulary(path, k: int = 10, L: int = 3, seed: int = 0, scoring: int = 0,
                     weighting: int = 0, flip: float = 0.25, stop_frac: float = 0.02):
    """A synthetic DBoW2 text vocabulary (ORBvoc.txt format: "k L scoring weighting", then
    "parent isLeaf d0..d31 weight" per node, breadth-first).  Children descriptors are noisy
    copies of their parent's, so descriptors descend meaningfully; leaf weights are
    idf-like positives with a few stop words (weight 0).  Returns the node count."""
    rng = np.random.default_rng(seed)
    lines = [f"{k} {L} {scoring} {weighting}"]
    desc = {0: rng.integers(0, 256, 32, dtype=np.uint8)}
    frontier, nid = [0], 1
    for level in range(1, L + 1):
        nxt = []
        for p in frontier:
            for _ in range(k):
                bits = rng.random(256) < flip
                d = desc[p] ^ np.packbits(bits, bitorder="little")
                desc[nid] = d
                leaf = level == L
                w = 0.0 if leaf and rng.random() < stop_frac else (
                    float(np.round(rng.uniform(0.5, 8.0), 6)) if leaf else 0.0)
                lines.append(f"{p} {int(leaf)} " + " ".join(str(int(b)) for b in d) + f" {w}")
                nxt.append(nid)
                nid += 1
        frontier = nxt
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return nid


# ---- keyframe database scenes (KeyFrameDatabase, src/KeyFrameDatabase.cc) --------------------

def _l1(values):
    v = np.asarray(values, np.float64)
    return v / v.sum() if len(v) else v


def kfdb_scene(seed: int, n_kf: int = 2000, vocab: int = 100000, words: int = 300,
               place: int = 600, window: int = 6, revisit: int = 0):
    """A synthetic keyframe trajectory for the keyframe database: keyframe t draws 75 % of its
    BowVector words from the word pool of its place (places drift along the trajectory, so
    neighbouring keyframes share many words) and 25 % at random; weights are L1-normalised like
    DBoW2's TF-IDF BowVectors.  With `revisit` > 0 the last `revisit` keyframes come back to the
    places of the first ones (loop-closure candidates far away in time).  The covisibility
    lists (KeyFrame::mvpOrderedConnectedKeyFrames) are the keyframes within `window` of t,
    ordered by shared-word count descending (ties by index descending, the reference's
    push_front of an ascending (weight, pointer) sort).  Returns (bows, covisibles, places)."""
    rng = np.random.default_rng(seed)
    n_places = max(2, n_kf // 4 + 2)
    pools = [rng.choice(vocab, place, replace=False) for _ in range(n_places)]
    place_of = np.minimum(np.arange(n_kf) // 4, n_places - 1)
    if revisit:
        place_of[n_kf - revisit:] = place_of[:revisit]
    bows = []
    for t in range(n_kf):
        p = place_of[t]
        own = rng.choice(pools[p], int(words * 0.75), replace=False)
        nxt = rng.choice(pools[min(p + 1, n_places - 1)], words // 10, replace=False)
        rnd = rng.choice(vocab, words - len(own) - len(nxt), replace=False)
        w = np.unique(np.concatenate([own, nxt, rnd])).astype(np.uint32)
        bows.append((w, _l1(rng.random(len(w)) + 0.05)))
    sets = [set(b[0].tolist()) for b in bows]
    cov = []
    for t in range(n_kf):
        cands = [u for u in range(max(0, t - window), min(n_kf, t + window + 1)) if u != t]
        wts = [(len(sets[t] & sets[u]), u) for u in cands]
        wts.sort()
        cov.append([u for _, u in reversed(wts)])
    return bows, cov, place_of


def kfdb_query(seed: int, bow, keep: float = 0.7, extra: int = 80, vocab: int = 100000):
    """A frame seen near a keyframe: `keep` of its words plus `extra` random words, weights
    re-drawn and L1-normalised."""
    rng = np.random.default_rng(seed)
    w = bow[0][rng.random(len(bow[0])) < keep]
    w = np.unique(np.concatenate([w, rng.choice(vocab, extra, replace=False)])).astype(np.uint32)
    return w, _l1(rng.random(len(w)) + 0.05)
