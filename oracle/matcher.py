"""ctypes front-end of the ORBmatcher restatement (oracle/orb_matcher_oracle.cpp).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Takes any object with the attributes of
my_orb_slam2_amd.features.FeatureSet (keys, desc, u_right, fvec, grid) and returns what the
reference methods return: the match count and per-feature indices.

Parity status: restatement of src/ORBmatcher.cc statement by statement; the reference has no
matcher fixtures and cannot be built here (OpenCV/DBoW2 absent), so it is pinned only by the
cross-checks in tests/ (PARITY UNPINNED against a run of the reference).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import lib as _lib_loader

_vp, _i, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float


class _FeatC(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("keys", _vp), ("desc", _vp), ("u_right", _vp),
                ("n_nodes", ctypes.c_int32), ("node_id", _vp), ("node_off", _vp),
                ("node_feat", _vp), ("grid_cols", ctypes.c_int32), ("grid_rows", ctypes.c_int32),
                ("grid_off", _vp), ("grid_feat", _vp), ("min_x", _f), ("min_y", _f),
                ("max_x", _f), ("max_y", _f), ("grid_inv_w", _f), ("grid_inv_h", _f)]


def _a(x):
    return None if x is None else x.ctypes.data


def _feat(fs) -> _FeatC:
    s = _FeatC()
    s.n = len(fs.keys)
    s.keys, s.desc, s.u_right = _a(fs.keys), _a(fs.desc), _a(fs.u_right)
    if fs.fvec is not None:
        s.n_nodes = len(fs.fvec.node_id)
        s.node_id, s.node_off, s.node_feat = _a(fs.fvec.node_id), _a(fs.fvec.off), _a(fs.fvec.feat)
    if fs.grid is not None:
        g = fs.grid
        s.grid_cols, s.grid_rows, s.grid_off, s.grid_feat = g.cols, g.rows, _a(g.off), _a(g.feat)
        s.min_x, s.min_y, s.max_x, s.max_y = g.min_x, g.min_y, g.max_x, g.max_y
        s.grid_inv_w, s.grid_inv_h = g.inv_w, g.inv_h
    return s


_L = None


def lib():
    global _L
    if _L is None:
        L = _lib_loader()
        L.oracle_three_maxima.argtypes = [_vp, _i, _vp]
        L.oracle_assign_grid.argtypes = [_vp, _i, _i, _i, _f, _f, _f, _f, _vp, _vp]
        L.oracle_search_by_bow_kf_frame.argtypes = [_vp, _vp, _vp, _f, _i, _vp]
        L.oracle_search_by_bow_kf_kf.argtypes = [_vp, _vp, _vp, _vp, _f, _i, _vp]
        L.oracle_search_for_triangulation.argtypes = [_vp, _vp, _vp, _vp, _vp, _f, _f, _vp, _vp,
                                                      _i, _i, _vp]
        L.oracle_search_by_projection.argtypes = [_i, _vp, _vp, _vp, _vp, _i, _vp, _i, _f, _i,
                                                  _vp]
        L.oracle_search_by_projection_ex.argtypes = [_i, _vp, _vp, _vp, _vp, _vp, _i, _vp, _i,
                                                     _f, _i, _i, _vp]
        L.oracle_search_by_sim3.argtypes = [_vp, _vp, _vp, _vp, _i, _vp, _vp, _i, _vp]
        L.oracle_search_for_initialization.argtypes = [_vp, _vp, _vp, _i, _f, _i, _vp]
        L.oracle_descriptor_distance_m.argtypes = [_vp, _vp]
        _L = L
    return _L


def _u8(m, n):
    return np.zeros(n, np.uint8) if m is None else np.ascontiguousarray(m).astype(np.uint8)


def three_maxima(counts):
    c = np.ascontiguousarray(counts, np.int32)
    out = np.zeros(3, np.int32)
    lib().oracle_three_maxima(_a(c), len(c), _a(out))
    return tuple(int(v) for v in out)


def assign_grid(keys, min_x, min_y, inv_w, inv_h, cols=64, rows=48):
    off = np.zeros(cols * rows + 1, np.int32)
    feat = np.zeros(max(len(keys), 1), np.int32)
    k = lib().oracle_assign_grid(_a(keys), len(keys), cols, rows, min_x, min_y, inv_w, inv_h,
                                 _a(off), _a(feat))
    return off, feat[:k]


def search_by_bow_kf_frame(kf, kf_valid, f, nnratio=0.6, check_ori=True):
    out = np.zeros(max(len(f.keys), 1), np.int32)
    a, b = _feat(kf), _feat(f)
    v = _u8(kf_valid, len(kf.keys))
    n = lib().oracle_search_by_bow_kf_frame(ctypes.byref(a), _a(v), ctypes.byref(b), nnratio,
                                            int(check_ori), _a(out))
    return n, out[:len(f.keys)]


def search_by_bow_kf_kf(k1, v1, k2, v2, nnratio=0.6, check_ori=True):
    out = np.zeros(max(len(k1.keys), 1), np.int32)
    a, b = _feat(k1), _feat(k2)
    m1, m2 = _u8(v1, len(k1.keys)), _u8(v2, len(k2.keys))
    n = lib().oracle_search_by_bow_kf_kf(ctypes.byref(a), _a(m1), ctypes.byref(b), _a(m2),
                                         nnratio, int(check_ori), _a(out))
    return n, out[:len(k1.keys)]


def search_for_triangulation(k1, has1, k2, has2, F12, epi, sigma2, scale, only_stereo=False,
                             check_ori=True):
    out = np.zeros(max(len(k1.keys), 1), np.int32)
    a, b = _feat(k1), _feat(k2)
    m1, m2 = _u8(has1, len(k1.keys)), _u8(has2, len(k2.keys))
    F = np.ascontiguousarray(F12, np.float32).reshape(9)
    s2 = np.ascontiguousarray(sigma2, np.float32)
    sc = np.ascontiguousarray(scale, np.float32)
    n = lib().oracle_search_for_triangulation(ctypes.byref(a), _a(m1), ctypes.byref(b), _a(m2),
                                              _a(F), float(epi[0]), float(epi[1]), _a(s2),
                                              _a(sc), int(only_stereo), int(check_ori), _a(out))
    m = out[:len(k1.keys)]
    idx1 = np.nonzero(m >= 0)[0]
    return n, np.stack([idx1, m[idx1]], axis=1).astype(np.int32)


def search_by_projection(mode, target, queries, qdesc, claimed=None, inv_sigma2=None,
                         orb_dist=0, nnratio=0.6, check_ori=True):
    q = np.ascontiguousarray(queries)
    d = np.ascontiguousarray(qdesc, np.uint8)
    out = np.zeros(max(len(q), 1), np.int32)
    t = _feat(target)
    cl = None if claimed is None else _u8(claimed, len(target.keys))
    isg = None if inv_sigma2 is None else np.ascontiguousarray(inv_sigma2, np.float32)
    n = lib().oracle_search_by_projection(int(mode), ctypes.byref(t), _a(cl), _a(d), _a(q),
                                          len(q), _a(isg), int(orb_dist), nnratio,
                                          int(check_ori), _a(out))
    return n, out[:len(q)]


def search_by_projection_ex(mode, target, queries, qdesc, qflags=None, claimed=None,
                            inv_sigma2=None, orb_dist=0, nnratio=0.6, check_ori=True,
                            prefilter=False):
    q = np.ascontiguousarray(queries)
    d = np.ascontiguousarray(qdesc, np.uint8)
    out = np.zeros(max(len(q), 1), np.int32)
    t = _feat(target)
    cl = None if claimed is None else _u8(claimed, len(target.keys))
    qf = None if qflags is None else _u8(qflags, len(q))
    isg = None if inv_sigma2 is None else np.ascontiguousarray(inv_sigma2, np.float32)
    n = lib().oracle_search_by_projection_ex(int(mode), ctypes.byref(t), _a(cl), _a(d), _a(q),
                                             _a(qf), len(q), _a(isg), int(orb_dist), nnratio,
                                             int(check_ori), int(prefilter), _a(out))
    return n, out[:len(q)]


def search_by_sim3(k1, k2, qdesc1, q12, qdesc2, q21):
    out = np.zeros(max(len(q12), 1), np.int32)
    a, b = _feat(k1), _feat(k2)
    q1, q2 = np.ascontiguousarray(q12), np.ascontiguousarray(q21)
    d1, d2 = np.ascontiguousarray(qdesc1, np.uint8), np.ascontiguousarray(qdesc2, np.uint8)
    n = lib().oracle_search_by_sim3(ctypes.byref(a), ctypes.byref(b), _a(d1), _a(q1), len(q1),
                                    _a(d2), _a(q2), len(q2), _a(out))
    return n, out[:len(q12)]


def search_for_initialization(f1, f2, prev_matched, window, nnratio=0.9, check_ori=True):
    out = np.zeros(max(len(f1.keys), 1), np.int32)
    a, b = _feat(f1), _feat(f2)
    assert prev_matched.dtype == np.float32 and prev_matched.flags.c_contiguous
    n = lib().oracle_search_for_initialization(ctypes.byref(a), ctypes.byref(b), _a(prev_matched),
                                               int(window), nnratio, int(check_ori), _a(out))
    return n, out[:len(f1.keys)]


def distinctive_descriptors(desc, off):
    """MapPoint::ComputeDistinctiveDescriptors restated, many points at once."""
    d = np.ascontiguousarray(desc, np.uint8)
    o = np.ascontiguousarray(off, np.int32)
    out = np.zeros(max(len(o) - 1, 1), np.int32)
    L = lib()
    L.oracle_distinctive_descriptors.argtypes = [_vp, _vp, _i, _vp]
    L.oracle_distinctive_descriptors(_a(d), _a(o), len(o) - 1, _a(out))
    return out[:len(o) - 1]


def bf_top2(q, db, r0=0, r1=None):
    """Brute-force Hamming top-2 restated (ORBmatcher's best / second loop over every row of
    db[r0:r1]); returns (best_idx, best_dist, second_dist) with global row numbers."""
    qa = np.ascontiguousarray(q, np.uint8).reshape(-1, 32)
    da = np.ascontiguousarray(db, np.uint8).reshape(-1, 32)
    r1 = len(da) if r1 is None else r1
    n = len(qa)
    bi = np.zeros(max(n, 1), np.int32)
    bd = np.zeros(max(n, 1), np.int32)
    sd = np.zeros(max(n, 1), np.int32)
    L = lib()
    L.oracle_bf_top2.argtypes = [_vp, _i, _vp, ctypes.c_longlong, ctypes.c_longlong, _vp, _vp, _vp]
    L.oracle_bf_top2(_a(qa), n, _a(da), r0, r1, _a(bi), _a(bd), _a(sd))
    return bi[:n], bd[:n], sd[:n]


class OracleVocabulary:
    """The DBoW2 restatement (oracle/orb_vocab_oracle.cpp)."""

    def __init__(self, path):
        L = lib()
        L.oracle_vocab_load.restype = _vp
        L.oracle_vocab_load.argtypes = [ctypes.c_char_p]
        L.oracle_vocab_free.argtypes = [_vp]
        L.oracle_vocab_transform.argtypes = [_vp, _vp, _i, _i] + [_vp] * 9
        L.oracle_bow_score_l1.restype = ctypes.c_double
        L.oracle_bow_score_l1.argtypes = [_vp, _vp, _i, _vp, _vp, _i]
        self._h = L.oracle_vocab_load(str(path).encode())
        if not self._h:
            raise ValueError(f"cannot load {path}")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_vocab_free(self._h)
            self._h = None

    def transform(self, desc, levelsup=4):
        d = np.ascontiguousarray(desc, np.uint8)
        n = len(d)
        cap = max(n, 1)
        word, node = np.zeros(cap, np.int32), np.zeros(cap, np.int32)
        bw, bv = np.zeros(cap, np.uint32), np.zeros(cap, np.float64)
        fn, fo, ff = np.zeros(cap, np.uint32), np.zeros(cap + 1, np.int32), np.zeros(cap, np.int32)
        nb, nf = ctypes.c_int32(), ctypes.c_int32()
        lib().oracle_vocab_transform(self._h, _a(d), n, levelsup, _a(word), _a(node),
                                     ctypes.byref(nb), _a(bw), _a(bv), ctypes.byref(nf), _a(fn),
                                     _a(fo), _a(ff))
        return (word[:n], node[:n], (bw[:nb.value], bv[:nb.value]),
                (fn[:nf.value], fo[:nf.value + 1], ff[:fo[nf.value]]))


def bow_score_l1(b1, b2):
    w1, v1 = np.ascontiguousarray(b1[0], np.uint32), np.ascontiguousarray(b1[1], np.float64)
    w2, v2 = np.ascontiguousarray(b2[0], np.uint32), np.ascontiguousarray(b2[1], np.float64)
    lib().oracle_bow_score_l1.restype = ctypes.c_double
    lib().oracle_bow_score_l1.argtypes = [_vp, _vp, _i, _vp, _vp, _i]
    return lib().oracle_bow_score_l1(_a(w1), _a(v1), len(w1), _a(w2), _a(v2), len(w2))


def undistort_keypoints(keys, K4, dist):
    """Frame::UndistortKeyPoints restated: returns the undistorted (x, y) float32 [n, 2]."""
    k = np.ascontiguousarray(K4, np.float32)
    d = np.ascontiguousarray(dist, np.float32)
    xy = np.ascontiguousarray(np.stack([keys["x"], keys["y"]], 1), np.float32)
    out = np.zeros_like(xy)
    L = lib()
    L.oracle_undistort_keypoints.argtypes = [_vp, _vp, _i, _vp, _i, _vp]
    L.oracle_undistort_keypoints(_a(k), _a(d), len(d), _a(xy), len(xy), _a(out))
    return out


def image_bounds(K4, dist, cols, rows):
    k = np.ascontiguousarray(K4, np.float32)
    d = np.ascontiguousarray(dist, np.float32)
    out = np.zeros(4, np.float32)
    L = lib()
    L.oracle_image_bounds.argtypes = [_vp, _vp, _i, _i, _i, _vp]
    L.oracle_image_bounds(_a(k), _a(d), len(d), cols, rows, _a(out))
    return tuple(float(v) for v in out)


def cvt_gray(img, rgb):
    s = np.ascontiguousarray(img, np.uint8)
    h, w, c = s.shape
    out = np.zeros((h, w), np.uint8)
    L = lib()
    L.oracle_cvt_gray.argtypes = [_vp, _i, _i, _i, _i, _vp]
    L.oracle_cvt_gray(_a(s), w, h, c, int(rgb), _a(out))
    return out


def is_in_frustum(frame, mps, skip=None, viewing_cos_limit=0.5, th=1.0):
    """Tracking::SearchLocalPoints' projection loop restated (Frame::isInFrustum +
    MapPoint::PredictScale + the SearchByProjection window, oracle/orb_frame_oracle.cpp):
    frame is one orbx_frame_pose record, mps orbx_map_point records (numpy structured arrays
    of my_orb_slam2_amd.features' dtypes).  Returns (queries as uint8 bytes of
    orbx_proj_query records, nToMatch)."""
    fr = np.ascontiguousarray(frame)
    m = np.ascontiguousarray(mps)
    sk = None if skip is None else np.ascontiguousarray(skip, np.uint8)
    q = np.zeros(len(m) * 32, np.uint8)
    L = lib()
    L.oracle_is_in_frustum.argtypes = [_vp, _vp, _i, _vp, _f, _f, _vp]
    L.oracle_is_in_frustum.restype = _i
    n = L.oracle_is_in_frustum(_a(fr), _a(m), len(m), _a(sk), viewing_cos_limit, th, _a(q))
    return q, n
