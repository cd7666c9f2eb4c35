"""ORBmatcher over liborbx.so (include/ORBmatcher.h:37-128, src/ORBmatcher.cc).

Method names follow the reference; arguments are the arrays the reference reads from its
Frame / KeyFrame / MapPoint objects (``FeatureSet``, masks, projected queries — see
include/orbx_match.h), results are feature indices (-1 = none) plus the reference's return
value.  Every call runs on the GPU; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, load, ptr
from .features import (PROJ_FRAME_MAPPOINTS, PROJ_FUSE, PROJ_FUSE_SCW, PROJ_KEYFRAME,
                       PROJ_KF_SCW, PROJ_LAST_FRAME, PROJ_QUERY_DTYPE, FeatureSet, featureset_c)

TH_LOW = 50      # src/ORBmatcher.cc:38
TH_HIGH = 100    # src/ORBmatcher.cc:37
HISTO_LENGTH = 30  # src/ORBmatcher.cc:39


def descriptor_distance(a: np.ndarray, b: np.ndarray) -> int:
    """ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1715-1731)."""
    a = np.ascontiguousarray(a, np.uint8).reshape(32)
    b = np.ascontiguousarray(b, np.uint8).reshape(32)
    return int(load().orbx_descriptor_distance(ptr(a), ptr(b)))


def compute_three_maxima(histo_counts) -> tuple[int, int, int]:
    """ORBmatcher::ComputeThreeMaxima (src/ORBmatcher.cc:1669-1710) on bin counts."""
    h = np.ascontiguousarray(histo_counts, np.int32)
    out = [ctypes.c_int32(-1) for _ in range(3)]
    load().orbx_compute_three_maxima(ptr(h), len(h), *[ctypes.byref(o) for o in out])
    return tuple(o.value for o in out)


class MatcherParams(ctypes.Structure):
    _fields_ = [("nnratio", ctypes.c_float), ("check_orientation", ctypes.c_int32),
                ("device", ctypes.c_int32)]


class KfDbC(ctypes.Structure):
    """orbx_kf_db (include/orbx_match.h) — device pointers."""
    _fields_ = [("nkf", ctypes.c_int32), ("max_feat", ctypes.c_int32),
                ("feat_off", ctypes.c_void_p), ("keys", ctypes.c_void_p),
                ("desc", ctypes.c_void_p), ("u_right", ctypes.c_void_p),
                ("flag", ctypes.c_void_p), ("node_off", ctypes.c_void_p),
                ("node_id", ctypes.c_void_p), ("node_feat_off", ctypes.c_void_p),
                ("node_feat", ctypes.c_void_p), ("node_keys", ctypes.c_void_p),
                ("node_desc", ctypes.c_void_p), ("node_u_right", ctypes.c_void_p),
                ("node_flag", ctypes.c_void_p)]


def _u8(mask, n):
    if mask is None:
        return np.zeros(n, np.uint8)
    m = np.ascontiguousarray(mask).astype(np.uint8, copy=False).reshape(-1)
    if len(m) != n:
        raise ValueError(f"mask has {len(m)} entries, expected {n}")
    return m


def _queries(q) -> np.ndarray:
    q = np.ascontiguousarray(q)
    if q.dtype != PROJ_QUERY_DTYPE:
        raise TypeError("queries must be a PROJ_QUERY_DTYPE array")
    return q


class ORBmatcher:
    """ORB_SLAM2::ORBmatcher(nnratio, checkOri) (src/ORBmatcher.cc:41-43)."""

    TH_LOW = TH_LOW
    TH_HIGH = TH_HIGH
    HISTO_LENGTH = HISTO_LENGTH
    DescriptorDistance = staticmethod(descriptor_distance)
    ComputeThreeMaxima = staticmethod(compute_three_maxima)

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, device: int = 0):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        self.device = int(device)
        self._lib = load()
        p = MatcherParams(self.mfNNratio, int(self.mbCheckOrientation), self.device)
        h = ctypes.c_void_p()
        check("orbx_matcher_create", self._lib.orbx_matcher_create(ctypes.byref(p),
                                                                   ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.orbx_matcher_destroy(h)
            self._h = None

    # ---- SearchByBoW ------------------------------------------------------------------
    def SearchByBoW(self, kf: FeatureSet, kf_valid, f: FeatureSet, f_valid=None,
                    f_is_keyframe: bool = False):
        """SearchByBoW(KeyFrame*, Frame&) (:182-319) -> (nmatches, KF index per F feature);
        with f_is_keyframe, SearchByBoW(KeyFrame*, KeyFrame*) (:563-696) ->
        (nmatches, KF2 index per KF1 feature)."""
        if f_is_keyframe:
            return self.search_by_bow_kf_kf(kf, kf_valid, f, f_valid)
        return self.search_by_bow_kf_frame(kf, kf_valid, f)

    def search_by_bow_kf_frame(self, kf: FeatureSet, kf_valid, f: FeatureSet):
        a, b = featureset_c(kf), featureset_c(f)
        va = _u8(kf_valid, kf.n)
        out = np.full(max(f.n, 1), -1, np.int32)
        n = ctypes.c_int32()
        check("orbx_search_by_bow_kf_frame", self._lib.orbx_search_by_bow_kf_frame(
            self._h, ctypes.byref(a), ptr(va), ctypes.byref(b), ptr(out), ctypes.byref(n)))
        return n.value, out[:f.n]

    def search_by_bow_kf_kf(self, kf1: FeatureSet, valid1, kf2: FeatureSet, valid2):
        a, b = featureset_c(kf1), featureset_c(kf2)
        v1, v2 = _u8(valid1, kf1.n), _u8(valid2, kf2.n)
        out = np.full(max(kf1.n, 1), -1, np.int32)
        n = ctypes.c_int32()
        check("orbx_search_by_bow_kf_kf", self._lib.orbx_search_by_bow_kf_kf(
            self._h, ctypes.byref(a), ptr(v1), ctypes.byref(b), ptr(v2), ptr(out),
            ctypes.byref(n)))
        return n.value, out[:kf1.n]

    # ---- SearchForTriangulation ---------------------------------------------------------
    def SearchForTriangulation(self, kf1: FeatureSet, has_mp1, kf2: FeatureSet, has_mp2, F12,
                               epipole, sigma2, scale, bOnlyStereo: bool = False):
        """(:702-872) -> (nmatches, pairs int32 [m, 2] of (idx1, idx2) in idx1 order)."""
        a, b = featureset_c(kf1), featureset_c(kf2)
        m1, m2 = _u8(has_mp1, kf1.n), _u8(has_mp2, kf2.n)
        F = np.ascontiguousarray(F12, np.float32).reshape(9)
        s2 = np.ascontiguousarray(sigma2, np.float32)
        sc = np.ascontiguousarray(scale, np.float32)
        cap = max(kf1.n, 1)
        pairs = np.zeros((cap, 2), np.int32)
        n = ctypes.c_int32()
        check("orbx_search_for_triangulation", self._lib.orbx_search_for_triangulation(
            self._h, ctypes.byref(a), ptr(m1), ctypes.byref(b), ptr(m2), ptr(F),
            float(epipole[0]), float(epipole[1]), ptr(s2), ptr(sc), len(s2), int(bOnlyStereo),
            ptr(pairs), cap, ctypes.byref(n)))
        return n.value, pairs[:n.value].copy()

    # ---- projection searches -------------------------------------------------------------
    def search_by_projection(self, mode: int, target: FeatureSet, queries, qdesc,
                             claimed=None, inv_sigma2=None, orb_dist: int = 0):
        """One of the projection searches (orbx_proj_mode) -> (nmatches, target index per
        query)."""
        q = _queries(queries)
        d = np.ascontiguousarray(qdesc, np.uint8).reshape(-1, 32)
        if len(d) != len(q):
            raise ValueError("one descriptor per query")
        t = featureset_c(target)
        cl = None if claimed is None else _u8(claimed, target.n)
        isg = None if inv_sigma2 is None else np.ascontiguousarray(inv_sigma2, np.float32)
        out = np.full(max(len(q), 1), -1, np.int32)
        n = ctypes.c_int32()
        check("orbx_search_by_projection", self._lib.orbx_search_by_projection(
            self._h, int(mode), ctypes.byref(t), ptr(cl), ptr(d), ptr(q), len(q), ptr(isg),
            0 if isg is None else len(isg), int(orb_dist), ptr(out), ctypes.byref(n)))
        return n.value, out[:len(q)]

    def search_by_projection_ex(self, mode: int, target: FeatureSet, queries, qdesc,
                                qflags=None, claimed=None, inv_sigma2=None, orb_dist: int = 0,
                                prefilter: bool = False):
        """orbx_search_by_projection_ex: per-query ORBX_QF_* flags (qflags) and the
        ORBX_PROJ_PREFILTER call flag -> (nmatches, target index per query)."""
        q = _queries(queries)
        d = np.ascontiguousarray(qdesc, np.uint8).reshape(-1, 32)
        if len(d) != len(q):
            raise ValueError("one descriptor per query")
        t = featureset_c(target)
        cl = None if claimed is None else _u8(claimed, target.n)
        qf = None if qflags is None else _u8(qflags, len(q))
        isg = None if inv_sigma2 is None else np.ascontiguousarray(inv_sigma2, np.float32)
        out = np.full(max(len(q), 1), -1, np.int32)
        n = ctypes.c_int32()
        check("orbx_search_by_projection_ex", self._lib.orbx_search_by_projection_ex(
            self._h, int(mode), ctypes.byref(t), ptr(cl), ptr(d), ptr(q), ptr(qf), len(q),
            ptr(isg), 0 if isg is None else len(isg), int(orb_dist), int(bool(prefilter)),
            ptr(out), ctypes.byref(n)))
        return n.value, out[:len(q)]

    def SearchByProjection(self, target: FeatureSet, queries, qdesc, claimed=None,
                           variant: str = "mappoints", orb_dist: int = TH_HIGH):
        """The four SearchByProjection overloads: variant "mappoints" (:46-132), "kf_scw"
        (:321-434), "last_frame" (:1392-1538), "keyframe" (:1540-1667)."""
        mode = {"mappoints": PROJ_FRAME_MAPPOINTS, "kf_scw": PROJ_KF_SCW,
                "last_frame": PROJ_LAST_FRAME, "keyframe": PROJ_KEYFRAME}[variant]
        return self.search_by_projection(mode, target, queries, qdesc, claimed,
                                         orb_dist=orb_dist)

    def Fuse(self, kf: FeatureSet, queries, qdesc, inv_sigma2=None, scw: bool = False):
        """Fuse(KeyFrame*, vpMapPoints, th) (:879-1029) or, with scw, Fuse(KeyFrame*, Scw, ...)
        (:1033-1156): the keyframe feature each MapPoint fuses with (the caller applies
        Replace / AddMapPoint in query order)."""
        mode = PROJ_FUSE_SCW if scw else PROJ_FUSE
        return self.search_by_projection(mode, kf, queries, qdesc, None, inv_sigma2)

    def SearchBySim3(self, kf1: FeatureSet, kf2: FeatureSet, qdesc1, q12, qdesc2, q21):
        """(:1158-1382) -> (nFound, KF2 index per KF1 feature)."""
        a, b = featureset_c(kf1), featureset_c(kf2)
        q1, q2 = _queries(q12), _queries(q21)
        d1 = np.ascontiguousarray(qdesc1, np.uint8).reshape(-1, 32)
        d2 = np.ascontiguousarray(qdesc2, np.uint8).reshape(-1, 32)
        out = np.full(max(len(q1), 1), -1, np.int32)
        n = ctypes.c_int32()
        check("orbx_search_by_sim3", self._lib.orbx_search_by_sim3(
            self._h, ctypes.byref(a), ctypes.byref(b), ptr(d1), ptr(q1), len(q1), ptr(d2),
            ptr(q2), len(q2), ptr(out), ctypes.byref(n)))
        return n.value, out[:len(q1)]

    def SearchForInitialization(self, f1: FeatureSet, f2: FeatureSet, prev_matched,
                                windowSize: int = 10):
        """(:446-561) -> (nmatches, vnMatches12); prev_matched (float32 [n1, 2]) is updated
        in place like vbPrevMatched."""
        a, b = featureset_c(f1), featureset_c(f2)
        if not (isinstance(prev_matched, np.ndarray) and prev_matched.dtype == np.float32
                and prev_matched.flags.c_contiguous and prev_matched.shape == (f1.n, 2)):
            raise TypeError("prev_matched must be a C-contiguous float32 array [n1, 2]")
        out = np.full(max(f1.n, 1), -1, np.int32)
        n = ctypes.c_int32()
        check("orbx_search_for_initialization", self._lib.orbx_search_for_initialization(
            self._h, ctypes.byref(a), ctypes.byref(b), ptr(prev_matched), int(windowSize),
            ptr(out), ctypes.byref(n)))
        return n.value, out[:f1.n]

    # ---- MapPoint::ComputeDistinctiveDescriptors ------------------------------------------
    def compute_distinctive_descriptors(self, desc, off):
        """MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:252-313) for many map points:
        point p's observed descriptors are rows off[p]..off[p+1] of desc; returns the chosen
        row per point (relative to off[p]), -1 for points without descriptors."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        o = np.ascontiguousarray(off, np.int32)
        best = np.full(max(len(o) - 1, 1), -1, np.int32)
        check("orbx_compute_distinctive_descriptors",
              self._lib.orbx_compute_distinctive_descriptors(self._h, ptr(d), ptr(o), len(o) - 1,
                                                              ptr(best)))
        return best[:len(o) - 1]

    BF_MFMA, BF_VALU = 0, 1

    def set_bf_kernel(self, kernel):
        """The brute-force top-2's distance kernel: BF_MFMA (k_bf_mfma, the default) or BF_VALU
        (k_bf_top2: v_xor + v_bcnt); the results are identical."""
        check("orbx_matcher_set_bf_kernel", self._lib.orbx_matcher_set_bf_kernel(self._h, int(kernel)))

    def hamming_bf_top2(self, q, db):
        """Brute-force Hamming top-2 of every query row against every database row, with the
        best / second loop of the ORBmatcher searches (src/ORBmatcher.cc:232-256): returns
        (best_idx, best_dist, second_dist), best_idx -1 where no row is below distance 256."""
        qa = np.ascontiguousarray(q, np.uint8).reshape(-1, 32)
        da = np.ascontiguousarray(db, np.uint8).reshape(-1, 32)
        n = len(qa)
        bi = np.full(max(n, 1), -1, np.int32)
        bd = np.full(max(n, 1), 256, np.int32)
        sd = np.full(max(n, 1), 256, np.int32)
        check("orbx_hamming_bf_top2",
              self._lib.orbx_hamming_bf_top2(self._h, ptr(qa), n, ptr(da), len(da), ptr(bi),
                                             ptr(bd), ptr(sd)))
        return bi[:n], bd[:n], sd[:n]

    def hamming_bf_top2_device(self, d_q, nq, d_db, ndb, d_best_idx, d_best_dist, d_second_dist,
                               idx_base=0, stream=0):
        """The same on device arrays (e.g. torch tensors) on `stream`; best_idx is offset by
        idx_base, so a shard of a larger database reports global rows (distributed.merge_top2
        folds the shards' results in shard order)."""
        check("orbx_hamming_bf_top2_device",
              self._lib.orbx_hamming_bf_top2_device(self._h, ptr(d_q), int(nq), ptr(d_db),
                                                    int(ndb), int(idx_base), ptr(d_best_idx),
                                                    ptr(d_best_dist), ptr(d_second_dist),
                                                    ctypes.c_void_p(stream)))

    # ---- batched device path ---------------------------------------------------------------
    def search_by_bow_kf_frame_batch_device(self, db: KfDbC, frame_c, d_match, d_nmatches,
                                            stream=0):
        """SearchByBoW(KeyFrame*, Frame&) of every keyframe of a device database against one
        device-resident frame (Tracking::Relocalization's candidate loop)."""
        check("orbx_search_by_bow_kf_frame_batch_device",
              self._lib.orbx_search_by_bow_kf_frame_batch_device(
                  self._h, ctypes.byref(db), ctypes.byref(frame_c), ptr(d_match),
                  ptr(d_nmatches), ctypes.c_void_p(stream)))

    def search_for_triangulation_batch_device(self, db: KfDbC, kf1, kf2, F12, epi, sigma2,
                                              scale, job_off, d_match, d_nmatches,
                                              only_stereo=False, stream=0):
        s2 = np.ascontiguousarray(sigma2, np.float32)
        sc = np.ascontiguousarray(scale, np.float32)
        check("orbx_search_for_triangulation_batch_device",
              self._lib.orbx_search_for_triangulation_batch_device(
                  self._h, ctypes.byref(db), int(kf1.numel()), ptr(kf1), ptr(kf2), ptr(F12),
                  ptr(epi), ptr(s2), ptr(sc), len(s2), int(only_stereo), ptr(job_off),
                  ptr(d_match), ptr(d_nmatches), ctypes.c_void_p(stream)))

    def search_by_projection_batch_device(self, mode: int, frames: "DeviceFrameBatch", d_qdesc,
                                          d_q, d_q_off, d_match, d_nmatches, d_claimed=None,
                                          inv_sigma2=None, orb_dist: int = 0, stream=0):
        """orbx_search_by_projection_batch_device: one projection search per frame of
        `frames`, queries of frame j at [d_q_off[j], d_q_off[j+1]) (device tensors)."""
        isg = None if inv_sigma2 is None else np.ascontiguousarray(inv_sigma2, np.float32)
        nq = int(d_q.numel() * d_q.element_size() // PROJ_QUERY_DTYPE.itemsize)
        check("orbx_search_by_projection_batch_device",
              self._lib.orbx_search_by_projection_batch_device(
                  self._h, int(mode), ctypes.byref(frames.c), frames.njobs, ptr(frames.feat_off),
                  ptr(frames.grid_pos_off), frames.max_feat, ptr(d_claimed), ptr(d_qdesc),
                  ptr(d_q), ptr(d_q_off), nq, ptr(isg), 0 if isg is None else len(isg),
                  int(orb_dist), ptr(d_match), ptr(d_nmatches), ctypes.c_void_p(stream)))

    def sync(self, stream=0):
        check("orbx_matcher_sync", self._lib.orbx_matcher_sync(self._h, ctypes.c_void_p(stream)))

    def profile(self, on: bool = True):
        check("orbx_matcher_profile_enable", self._lib.orbx_matcher_profile_enable(self._h, int(on)))

    def collect_profile(self) -> dict:
        from ._lib import MATCH_KERNELS
        ms = np.zeros(len(MATCH_KERNELS), np.float64)
        cnt = np.zeros(len(MATCH_KERNELS), np.int64)
        check("orbx_matcher_profile_collect",
              self._lib.orbx_matcher_profile_collect(self._h, ptr(ms), ptr(cnt)))
        return {k: (float(ms[i]), int(cnt[i])) for i, k in enumerate(MATCH_KERNELS)}


class DeviceFeatureSet:
    """A FeatureSet copied to device memory (torch tensors) with its orbx_featureset view."""

    def __init__(self, fs: FeatureSet, device):
        import torch
        from .features import FeatureSetC

        def t(a, dtype=None):
            a = np.ascontiguousarray(a if dtype is None else a.astype(dtype))
            return torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to(device)

        n = fs.n
        self.keys = t(fs.keys) if n else torch.zeros(28, dtype=torch.uint8, device=device)
        self.desc = t(fs.desc) if n else torch.zeros(32, dtype=torch.uint8, device=device)
        ur = fs.u_right if fs.u_right is not None else np.full(n, -1.0, np.float32)
        self.u_right = t(np.ascontiguousarray(ur, np.float32)) if n else None
        fv = fs.fvec
        self.node_id = t(fv.node_id) if fv is not None and len(fv.node_id) else None
        self.node_off = t(fv.off) if fv is not None else None
        self.node_feat = t(fv.feat) if fv is not None and len(fv.feat) else None
        c = FeatureSetC()
        c.n = n
        c.keys, c.desc = self.keys.data_ptr(), self.desc.data_ptr()
        c.u_right = self.u_right.data_ptr() if self.u_right is not None else None
        if fv is not None and len(fv.node_id):
            c.n_nodes = len(fv.node_id)
            c.node_id, c.node_off = self.node_id.data_ptr(), self.node_off.data_ptr()
            c.node_feat = self.node_feat.data_ptr()
        self.c = c


class DeviceFrameBatch:
    """Frames (FeatureSets with grids of one camera) concatenated in device memory for
    orbx_search_by_projection_batch_device."""

    def __init__(self, featuresets, device):
        import torch
        from .features import FeatureSetC
        fss = list(featuresets)
        g0 = fss[0].grid
        for fs in fss:
            g = fs.grid
            if (g.cols, g.rows, g.min_x, g.min_y, g.inv_w, g.inv_h) != (
                    g0.cols, g0.rows, g0.min_x, g0.min_y, g0.inv_w, g0.inv_h):
                raise ValueError("frames of one batch share the grid geometry")
        self.njobs = len(fss)
        n = np.array([fs.n for fs in fss], np.int64)
        feat_off = np.zeros(len(fss) + 1, np.int32)
        np.cumsum(n, out=feat_off[1:])
        gn = np.array([len(fs.grid.feat) for fs in fss], np.int64)
        gpos = np.zeros(len(fss) + 1, np.int32)
        np.cumsum(gn, out=gpos[1:])
        self.max_feat = int(n.max())

        def t(a, dtype=None):
            a = np.ascontiguousarray(a if dtype is None else a.astype(dtype))
            b = a.view(np.uint8).reshape(-1) if a.size else np.zeros(16, np.uint8)
            return torch.from_numpy(b.copy()).to(device)

        self.keys = t(np.concatenate([fs.keys for fs in fss]))
        self.desc = t(np.concatenate([fs.desc for fs in fss]))
        self.u_right = t(np.concatenate([fs.u_right if fs.u_right is not None else
                                         np.full(fs.n, -1.0, np.float32) for fs in fss]),
                         np.float32)
        self.grid_off = t(np.concatenate([fs.grid.off for fs in fss]), np.int32)
        self.grid_feat = t(np.concatenate([fs.grid.feat for fs in fss]), np.int32)
        self.feat_off = torch.from_numpy(feat_off).to(device)
        self.grid_pos_off = torch.from_numpy(gpos).to(device)
        self.h_feat_off = feat_off
        c = FeatureSetC()
        c.n = int(feat_off[-1])
        c.keys, c.desc = self.keys.data_ptr(), self.desc.data_ptr()
        c.u_right = self.u_right.data_ptr()
        c.grid_cols, c.grid_rows = g0.cols, g0.rows
        c.grid_off, c.grid_feat = self.grid_off.data_ptr(), self.grid_feat.data_ptr()
        c.min_x, c.min_y, c.max_x, c.max_y = g0.min_x, g0.min_y, g0.max_x, g0.max_y
        c.grid_inv_w, c.grid_inv_h = g0.inv_w, g0.inv_h
        self.c = c


class DeviceKfDb:
    """A keyframe database (orbx_kf_db) in device memory: the FeatureSets concatenated, with
    per-keyframe MapPoint flags (valid for BoW, has_mp for triangulation)."""

    def __init__(self, featuresets, flags, device):
        import torch
        fss = list(featuresets)
        n = np.array([fs.n for fs in fss], np.int64)
        feat_off = np.zeros(len(fss) + 1, np.int32)
        np.cumsum(n, out=feat_off[1:])
        keys = np.concatenate([fs.keys for fs in fss]) if len(fss) else np.zeros(0)
        desc = np.concatenate([fs.desc for fs in fss]) if len(fss) else np.zeros((0, 32), np.uint8)
        ur = np.concatenate([fs.u_right if fs.u_right is not None else
                             np.full(fs.n, -1.0, np.float32) for fs in fss]).astype(np.float32)
        fl = np.concatenate([np.asarray(f, np.uint8).reshape(-1) for f in flags]).astype(np.uint8)
        nn = np.array([len(fs.fvec.node_id) for fs in fss], np.int64)
        node_off = np.zeros(len(fss) + 1, np.int32)
        np.cumsum(nn, out=node_off[1:])
        node_id = np.concatenate([fs.fvec.node_id for fs in fss]).astype(np.uint32)
        nfo, nf, base = [], [], 0
        for fs in fss:
            o = fs.fvec.off
            nfo.append(o[:-1] - o[0] + base)
            nf.append(fs.fvec.feat[o[0]:o[-1]])
            base += int(o[-1] - o[0])
        node_feat_off = np.concatenate(nfo + [np.array([base])]).astype(np.int32)
        node_feat = np.concatenate(nf).astype(np.int32) if nf else np.zeros(0, np.int32)

        def t(a):
            a = np.ascontiguousarray(a)
            b = a.view(np.uint8).reshape(-1) if a.size else np.zeros(16, np.uint8)
            return torch.from_numpy(b.copy()).to(device)

        self.tensors = [t(feat_off), t(keys), t(desc), t(ur), t(fl), t(node_off), t(node_id),
                        t(node_feat_off), t(node_feat)]
        p = [x.data_ptr() for x in self.tensors]
        self.c = KfDbC(len(fss), int(n.max()) if len(fss) else 0, *p)
        self.feat_off = feat_off
        self.n_entries = int(base)
        self._device = device

    def node_order(self, matcher, stream=0):
        """Give the database its node-order copies (orbx_kf_db_node_order): the per-node
        matchers (SearchForTriangulation) then read contiguous runs instead of gathering each
        feature.  Returns self."""
        import torch
        n = max(self.n_entries, 1)
        self.node_tensors = [torch.empty(n * 28, dtype=torch.uint8, device=self._device),
                             torch.empty(n * 32, dtype=torch.uint8, device=self._device),
                             torch.empty(n, dtype=torch.float32, device=self._device),
                             torch.empty(n, dtype=torch.uint8, device=self._device)]
        k, d, u, f = (x.data_ptr() for x in self.node_tensors)
        check("orbx_kf_db_node_order", matcher._lib.orbx_kf_db_node_order(
            matcher._h, ctypes.byref(self.c), self.n_entries, ctypes.c_void_p(k),
            ctypes.c_void_p(d), ctypes.c_void_p(u), ctypes.c_void_p(f), ctypes.c_void_p(stream)))
        self.c.node_keys, self.c.node_desc, self.c.node_u_right, self.c.node_flag = k, d, u, f
        return self
