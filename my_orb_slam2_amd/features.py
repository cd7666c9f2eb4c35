"""Per-frame feature arrays the matchers read (the POD view of Frame / KeyFrame).

``FeatureSet`` holds what ORBmatcher touches on a Frame or KeyFrame (src/Frame.h,
src/KeyFrame.h): mvKeysUn, mDescriptors, mvuRight, mFeatVec and mGrid.  The grid and the
FeatureVector are built here with the reference's host rules:

* ``assign_features_to_grid`` — Frame::AssignFeaturesToGrid + PosInGrid
  (src/Frame.cc:243-258, 407-417) with the cell size of Frame.cc:114-115 / 168-169 / 225-226
  (mfGridElementWidthInv = float(FRAME_GRID_COLS) / float(mnMaxX - mnMinX)).
* ``feature_vector`` — DBoW2::FeatureVector (Thirdparty/DBoW2/DBoW2/FeatureVector.cpp:31-45):
  std::map<NodeId, vector<feature index>>, features appended in extraction order.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from ._lib import KEYPOINT_DTYPE

FRAME_GRID_COLS = 64   # include/Frame.h:38
FRAME_GRID_ROWS = 48   # include/Frame.h:37


def round_half_away(v) -> np.ndarray:
    """std::round on float values (half away from zero), exactly, via float64."""
    v = np.asarray(v, np.float64)
    return (np.sign(v) * np.floor(np.abs(v) + 0.5)).astype(np.int64)


@dataclass
class Grid:
    cols: int
    rows: int
    off: np.ndarray        # int32 [cols*rows + 1], cell c = ix*rows + iy
    feat: np.ndarray       # int32
    min_x: float
    min_y: float
    max_x: float
    max_y: float
    inv_w: float
    inv_h: float


def assign_features_to_grid(keys: np.ndarray, min_x: float, max_x: float, min_y: float,
                            max_y: float, cols: int = FRAME_GRID_COLS,
                            rows: int = FRAME_GRID_ROWS) -> Grid:
    """Frame::AssignFeaturesToGrid (src/Frame.cc:243-258) as a CSR grid."""
    f32 = np.float32
    inv_w = f32(cols) / f32(f32(max_x) - f32(min_x))
    inv_h = f32(rows) / f32(f32(max_y) - f32(min_y))
    x = np.asarray(keys["x"], f32)
    y = np.asarray(keys["y"], f32)
    px = round_half_away((x - f32(min_x)) * inv_w)     # PosInGrid, Frame.cc:409-410
    py = round_half_away((y - f32(min_y)) * inv_h)
    ok = (px >= 0) & (px < cols) & (py >= 0) & (py < rows)
    idx = np.nonzero(ok)[0]
    cell = px[idx] * rows + py[idx]
    order = np.argsort(cell, kind="stable")            # within a cell: index order
    feat = idx[order].astype(np.int32)
    counts = np.bincount(cell, minlength=cols * rows)
    off = np.zeros(cols * rows + 1, np.int32)
    np.cumsum(counts, out=off[1:])
    return Grid(cols, rows, off, feat, float(f32(min_x)), float(f32(min_y)), float(f32(max_x)),
                float(f32(max_y)), float(inv_w), float(inv_h))


@dataclass
class FeatureVector:
    node_id: np.ndarray    # uint32, ascending
    off: np.ndarray        # int32 [n_nodes + 1]
    feat: np.ndarray       # int32


def feature_vector(node_of_feature: np.ndarray) -> FeatureVector:
    """FeatureVector from the node each feature was assigned to (-1 = none)."""
    nodes = np.asarray(node_of_feature, np.int64)
    idx = np.nonzero(nodes >= 0)[0]
    order = np.argsort(nodes[idx], kind="stable")
    feat = idx[order].astype(np.int32)
    ids, counts = np.unique(nodes[idx][order], return_counts=True)
    off = np.zeros(len(ids) + 1, np.int32)
    np.cumsum(counts, out=off[1:])
    return FeatureVector(ids.astype(np.uint32), off, feat)


@dataclass
class FeatureSet:
    """mvKeysUn / mDescriptors / mvuRight / mFeatVec / mGrid of one Frame or KeyFrame."""
    keys: np.ndarray                      # KEYPOINT_DTYPE [n]
    desc: np.ndarray                      # uint8 [n, 32]
    u_right: np.ndarray | None = None     # float32 [n] (None = monocular)
    fvec: FeatureVector | None = None
    grid: Grid | None = None
    _keep: list = field(default_factory=list, repr=False)

    def __post_init__(self):
        self.keys = np.ascontiguousarray(self.keys, KEYPOINT_DTYPE)
        self.desc = np.ascontiguousarray(self.desc, np.uint8).reshape(-1, 32)
        if self.u_right is not None:
            self.u_right = np.ascontiguousarray(self.u_right, np.float32)
        if len(self.keys) != len(self.desc):
            raise ValueError("keys and descriptors differ in length")

    @property
    def n(self) -> int:
        return len(self.keys)


class FeatureSetC(ctypes.Structure):
    """orbx_featureset (include/orbx_match.h)."""
    _fields_ = [("n", ctypes.c_int32), ("keys", ctypes.c_void_p), ("desc", ctypes.c_void_p),
                ("u_right", ctypes.c_void_p), ("n_nodes", ctypes.c_int32),
                ("node_id", ctypes.c_void_p), ("node_off", ctypes.c_void_p),
                ("node_feat", ctypes.c_void_p), ("grid_cols", ctypes.c_int32),
                ("grid_rows", ctypes.c_int32), ("grid_off", ctypes.c_void_p),
                ("grid_feat", ctypes.c_void_p), ("min_x", ctypes.c_float),
                ("min_y", ctypes.c_float), ("max_x", ctypes.c_float), ("max_y", ctypes.c_float),
                ("grid_inv_w", ctypes.c_float), ("grid_inv_h", ctypes.c_float)]


def _addr(a):
    return None if a is None else a.ctypes.data


def featureset_c(fs: FeatureSet) -> FeatureSetC:
    """The C view of a FeatureSet (host pointers; `fs` must outlive the struct)."""
    s = FeatureSetC()
    s.n = fs.n
    s.keys = _addr(fs.keys)
    s.desc = _addr(fs.desc)
    s.u_right = _addr(fs.u_right)
    if fs.fvec is not None:
        s.n_nodes = len(fs.fvec.node_id)
        s.node_id, s.node_off, s.node_feat = (_addr(fs.fvec.node_id), _addr(fs.fvec.off),
                                              _addr(fs.fvec.feat))
    if fs.grid is not None:
        g = fs.grid
        s.grid_cols, s.grid_rows = g.cols, g.rows
        s.grid_off, s.grid_feat = _addr(g.off), _addr(g.feat)
        s.min_x, s.min_y, s.max_x, s.max_y = g.min_x, g.min_y, g.max_x, g.max_y
        s.grid_inv_w, s.grid_inv_h = g.inv_w, g.inv_h
    return s


PROJ_QUERY_DTYPE = np.dtype([("u", "<f4"), ("v", "<f4"), ("ur", "<f4"), ("radius", "<f4"),
                             ("min_level", "<i4"), ("max_level", "<i4"),
                             ("pred_level", "<i4"), ("angle", "<f4")])

# orbx_proj_mode (include/orbx_match.h)
PROJ_FRAME_MAPPOINTS = 0
PROJ_KF_SCW = 1
PROJ_LAST_FRAME = 2
PROJ_KEYFRAME = 3
PROJ_FUSE = 4
PROJ_FUSE_SCW = 5
PROJ_SIM3 = 6


# ---- Frame geometry (include/orbx_frame.h) ------------------------------------------------

def _cam(K4, dist):
    k = np.ascontiguousarray(K4, np.float32).reshape(4)
    d = np.ascontiguousarray(dist, np.float32).reshape(-1)
    if len(d) not in (4, 5, 8):
        raise ValueError("distortion needs 4, 5 or 8 coefficients")
    return k, d


def undistort_keypoints(keys: np.ndarray, K4, dist, device: int = 0) -> np.ndarray:
    """Frame::UndistortKeyPoints (src/Frame.cc:429-459) on the GPU: mvKeysUn from mvKeys."""
    from ._lib import check, load, ptr
    k, d = _cam(K4, dist)
    src = np.ascontiguousarray(keys, KEYPOINT_DTYPE)
    out = src.copy()
    check("orbx_undistort_keypoints", load().orbx_undistort_keypoints(
        ptr(k), ptr(d), len(d), ptr(src), len(src), ptr(out), device))
    return out


def image_bounds(K4, dist, width: int, height: int):
    """Frame::ComputeImageBounds (src/Frame.cc:461-489) -> (minX, maxX, minY, maxY)."""
    from ._lib import check, load, ptr
    k, d = _cam(K4, dist)
    b = np.zeros(4, np.float32)
    check("orbx_image_bounds", load().orbx_image_bounds(ptr(k), ptr(d), len(d), width, height,
                                                         ptr(b)))
    return tuple(float(v) for v in b)


def assign_grid_device(d_keys, n: int, min_x: float, max_x: float, min_y: float, max_y: float,
                       d_off, d_feat, cols: int = FRAME_GRID_COLS, rows: int = FRAME_GRID_ROWS,
                       stream: int = 0):
    """Frame::AssignFeaturesToGrid on device keypoints (torch tensors) -> fills d_off
    (cols*rows + 1) and d_feat (n)."""
    from ._lib import check, load, ptr
    f32 = np.float32
    inv_w = f32(cols) / f32(f32(max_x) - f32(min_x))
    inv_h = f32(rows) / f32(f32(max_y) - f32(min_y))
    check("orbx_assign_grid_device", load().orbx_assign_grid_device(
        ptr(d_keys), n, cols, rows, float(f32(min_x)), float(f32(min_y)), float(inv_w),
        float(inv_h), ptr(d_off), ptr(d_feat), ctypes.c_void_p(stream)))


def assign_grid_batch_device(d_keys, kp_stride: int, d_n, batch: int, bounds, d_off, d_feat,
                             cols: int = FRAME_GRID_COLS, rows: int = FRAME_GRID_ROWS,
                             stream: int = 0):
    """AssignFeaturesToGrid for `batch` frames laid out like orbx_batch_view (device
    tensors): d_off [batch][cols*rows + 1], d_feat [batch][kp_stride].  bounds =
    (min_x, max_x, min_y, max_y)."""
    from ._lib import check, load, ptr
    f32 = np.float32
    min_x, max_x, min_y, max_y = (f32(b) for b in bounds)
    inv_w = f32(cols) / f32(max_x - min_x)
    inv_h = f32(rows) / f32(max_y - min_y)
    check("orbx_assign_grid_batch_device", load().orbx_assign_grid_batch_device(
        ptr(d_keys), int(kp_stride), ptr(d_n), int(batch), cols, rows, float(min_x),
        float(min_y), float(inv_w), float(inv_h), ptr(d_off), ptr(d_feat),
        ctypes.c_void_p(stream)))
    return float(inv_w), float(inv_h)


def undistort_keypoints_batch_device(K4, dist, d_keys, kp_stride: int, d_n, batch: int,
                                     d_out, stream: int = 0):
    """Frame::UndistortKeyPoints for `batch` frames laid out like orbx_batch_view."""
    from ._lib import check, load, ptr
    k = np.ascontiguousarray(K4, np.float32)
    d = np.ascontiguousarray(dist, np.float32)
    check("orbx_undistort_keypoints_batch_device", load().orbx_undistort_keypoints_batch_device(
        ptr(k), ptr(d), len(d), ptr(d_keys), int(kp_stride), ptr(d_n), int(batch), ptr(d_out),
        ctypes.c_void_p(stream)))


def cvt_color_gray(img: np.ndarray, rgb: bool = False, device: int = 0) -> np.ndarray:
    """Tracking's colour conversion (src/Tracking.cc:189-214): cvtColor(*2GRAY) of an 8-bit
    3- or 4-channel image on the GPU (rgb=True for RGB/RGBA order, mbRGB)."""
    from ._lib import check, load, ptr
    src = np.ascontiguousarray(img, np.uint8)
    if src.ndim != 3 or src.shape[2] not in (3, 4):
        raise ValueError("expected an H x W x 3 or H x W x 4 uint8 image")
    h, w, c = src.shape
    out = np.zeros((h, w), np.uint8)
    check("orbx_cvt_color", load().orbx_cvt_color(ptr(src), w, h, w * c, c, int(rgb), ptr(out),
                                                   w, device))
    return out


# ---- Frame::isInFrustum + MapPoint::PredictScale (include/orbx_frame.h) ---------------------

# orbx_map_point: GetWorldPos, mfMinDistance, GetNormal, mfMaxDistance (32 bytes)
MAP_POINT_DTYPE = np.dtype([("pos", "<f4", 3), ("min_dist", "<f4"), ("normal", "<f4", 3),
                            ("max_dist", "<f4")])
# orbx_frame_pose: mRcw (row-major), mtcw, mOw, fx fy cx cy mbf, image bounds,
# mfLogScaleFactor, mnScaleLevels, mvScaleFactors
FRAME_POSE_DTYPE = np.dtype([("Rcw", "<f4", 9), ("tcw", "<f4", 3), ("Ow", "<f4", 3),
                             ("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"), ("cy", "<f4"),
                             ("mbf", "<f4"), ("min_x", "<f4"), ("max_x", "<f4"),
                             ("min_y", "<f4"), ("max_y", "<f4"), ("log_scale_factor", "<f4"),
                             ("nlevels", "<i4"), ("scale", "<f4", 16)])


def frame_pose(Rcw, tcw, K4, bounds, scale_factors, mbf: float = 0.0,
               scale_factor: float = 1.2) -> np.ndarray:
    """One orbx_frame_pose record from a pose (Rcw, tcw): Ow = -Rcw^T tcw (the Frame's mOw,
    Frame::UpdatePoseMatrices, Frame.cc:271-278; the caller passes its own mOw, so only its
    value matters here), mfLogScaleFactor = logf(mfScaleFactor) (Frame.cc:82; for 1.2f the
    double log rounded to float is glibc's logf value, tests/test_frustum.py)."""
    import math
    f = np.zeros((), FRAME_POSE_DTYPE)
    R = np.asarray(Rcw, np.float32).reshape(3, 3)
    t = np.asarray(tcw, np.float32).reshape(3)
    f["Rcw"] = R.reshape(9)
    f["tcw"] = t
    f["Ow"] = (-(R.astype(np.float64).T @ t.astype(np.float64))).astype(np.float32)
    f["fx"], f["fy"], f["cx"], f["cy"] = (np.float32(v) for v in np.asarray(K4, np.float32))
    f["mbf"] = np.float32(mbf)
    f["min_x"], f["max_x"], f["min_y"], f["max_y"] = (np.float32(b) for b in bounds)
    sc = np.asarray(scale_factors, np.float32)
    f["nlevels"] = len(sc)
    f["scale"][:len(sc)] = sc
    f["log_scale_factor"] = np.float32(math.log(float(np.float32(scale_factor))))
    return f


def is_in_frustum(frame: np.ndarray, mps: np.ndarray, skip=None, viewing_cos_limit: float = 0.5,
                  th: float = 1.0, device: int = 0):
    """Tracking::SearchLocalPoints' projection of one frame's local map on the GPU
    (Frame::isInFrustum + PredictScale, Frame.cc:285-349, MapPoint.cc:430-444): returns the
    SearchByProjection queries (PROJ_QUERY_DTYPE, radius -1 = not in view) and nToMatch."""
    from ._lib import check, load, ptr
    fr = np.ascontiguousarray(frame, FRAME_POSE_DTYPE).reshape(())
    m = np.ascontiguousarray(mps, MAP_POINT_DTYPE)
    sk = None if skip is None else np.ascontiguousarray(skip, np.uint8)
    q = np.zeros(len(m), PROJ_QUERY_DTYPE)
    nv = ctypes.c_int32(0)
    check("orbx_is_in_frustum", load().orbx_is_in_frustum(
        ptr(fr), ptr(m), len(m), ptr(sk), float(viewing_cos_limit), float(th), ptr(q),
        ctypes.byref(nv), device))
    return q, nv.value


def is_in_frustum_batch_device(d_frames, nframes: int, d_mps, d_mp_off, max_mps: int, d_skip,
                               d_q, d_nvisible=None, viewing_cos_limit: float = 0.5,
                               th: float = 1.0, stream: int = 0):
    """The same for `nframes` frames on device arrays (torch tensors): frame f's MapPoints at
    [d_mp_off[f], d_mp_off[f+1]) of d_mps, queries into d_q at the same indices."""
    from ._lib import check, load, ptr
    check("orbx_is_in_frustum_batch_device", load().orbx_is_in_frustum_batch_device(
        ptr(d_frames), int(nframes), ptr(d_mps), ptr(d_mp_off), int(max_mps), ptr(d_skip),
        float(viewing_cos_limit), float(th), ptr(d_q), ptr(d_nvisible), ctypes.c_void_p(stream)))
