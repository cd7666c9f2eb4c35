"""Batched monocular tracking front-end: B frames per call, device-resident end to end.

Per frame, the reference's mono Tracking does (src/Tracking.cc):
  Frame::Frame (mono)      ExtractORB (Frame.cc:204), UndistortKeyPoints (:429-458),
                           AssignFeaturesToGrid (:243-258); image bounds once per camera
                           (ComputeImageBounds :461-489)
  SearchLocalPoints        Frame::isInFrustum + MapPoint::PredictScale on every local MapPoint
                           (Tracking.cc:1322-1335, Frame.cc:285-349, MapPoint.cc:430-444),
                           then ORBmatcher(0.8).SearchByProjection(mCurrentFrame,
                           mvpLocalMapPoints, th) (Tracking.cc:1337-1346, ORBmatcher.cc:41-136)

``MonoTrackBatch`` runs those stages for B frames on one HIP stream: one batched extraction
(orbx_extract_batch_device), one batched undistortion and grid pass (orbx_frame.h batch
forms), one batched projection of the frames' local maps (orbx_is_in_frustum_batch_device:
the pose, the MapPoints' positions, normals and distances in; the SearchByProjection queries
out) and one batched projection search (orbx_search_by_projection_batch_device) whose job j is
frame j.  ``search_local_points`` also takes ready-made queries (the caller's own projection).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import KEYPOINT_DTYPE, check
from .extractor import ORBextractor
from .features import (FRAME_GRID_COLS, FRAME_GRID_ROWS, PROJ_FRAME_MAPPOINTS, PROJ_QUERY_DTYPE,
                       FeatureSetC, assign_grid_batch_device, image_bounds,
                       is_in_frustum_batch_device, undistort_keypoints_batch_device)
from .matcher import ORBmatcher


class MonoTrackBatch:
    def __init__(self, batch: int, width: int, height: int, K4, dist, nfeatures: int = 1000,
                 scaleFactor: float = 1.2, nlevels: int = 8, iniThFAST: int = 20,
                 minThFAST: int = 7, nnratio: float = 0.8, device: int = 0):
        import torch
        self.batch, self.width, self.height = batch, width, height
        self.K4 = np.asarray(K4, np.float32)
        self.dist = np.asarray(dist, np.float32)
        self.dev = torch.device("cuda", device)
        self.ext = ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST,
                                max_batch=batch, device=device)
        self.kp_cap = self.ext.prepare(width, height, batch)
        self.matcher = ORBmatcher(nnratio, True, device=device)   # Tracking.cc:1338
        self.bounds = image_bounds(self.K4, self.dist, width, height)
        cells = FRAME_GRID_COLS * FRAME_GRID_ROWS
        kc = self.kp_cap
        self.keys_un = torch.empty(batch * kc * KEYPOINT_DTYPE.itemsize, dtype=torch.uint8,
                                   device=self.dev)
        self.grid_off = torch.empty((batch, cells + 1), dtype=torch.int32, device=self.dev)
        self.grid_feat = torch.empty((batch, kc), dtype=torch.int32, device=self.dev)
        offs = torch.arange(batch + 1, dtype=torch.int32, device=self.dev) * kc
        self.feat_off = offs            # frame j's slots [j*kp_cap, (j+1)*kp_cap)
        self.grid_pos_off = offs        # frame j's grid entries at j*kp_cap
        self.max_feat = kc
        self.njobs = batch
        self._c = None

    def _featureset(self):
        v = self.ext.batch_view()
        b = self.bounds
        inv_w = np.float32(FRAME_GRID_COLS) / np.float32(np.float32(b[1]) - np.float32(b[0]))
        inv_h = np.float32(FRAME_GRID_ROWS) / np.float32(np.float32(b[3]) - np.float32(b[2]))
        c = FeatureSetC()
        c.n = self.batch * self.kp_cap
        c.keys, c.desc, c.u_right = self.keys_un.data_ptr(), v.desc, None
        c.grid_cols, c.grid_rows = FRAME_GRID_COLS, FRAME_GRID_ROWS
        c.grid_off, c.grid_feat = self.grid_off.data_ptr(), self.grid_feat.data_ptr()
        c.min_x, c.max_x, c.min_y, c.max_y = b
        c.grid_inv_w, c.grid_inv_h = float(inv_w), float(inv_h)
        self.c = c
        return v

    def frames(self, images, stream: int = 0):
        """Frame construction for a [B, H, W] uint8 device tensor: extraction, undistortion and
        grid.  Returns the orbx_batch_view of the extraction."""
        B, H, W = images.shape
        if B != self.batch or (W, H) != (self.width, self.height):
            raise ValueError("batch shape differs from the prepared one")
        self.ext.extract_batch_device(images, stream)
        v = self._featureset()
        undistort_keypoints_batch_device(self.K4, self.dist, v.kps, self.kp_cap, v.nkp, B,
                                         self.keys_un, stream)
        assign_grid_batch_device(self.keys_un, self.kp_cap, v.nkp, B, self.bounds,
                                 self.grid_off, self.grid_feat, stream=stream)
        return v

    def search_local_points(self, d_qdesc, d_q, d_q_off, d_match, d_nmatches, d_claimed=None,
                            stream: int = 0):
        """SearchByProjection(Frame, local MapPoints) for every frame of the last ``frames``
        call: frame j's projected MapPoints at [d_q_off[j], d_q_off[j+1]) of d_q / d_qdesc;
        d_claimed (B * kp_cap bytes) marks features already matched by the motion-model
        search (mvpMapPoints set, ORBmatcher.cc:90-92)."""
        self.matcher.search_by_projection_batch_device(
            PROJ_FRAME_MAPPOINTS, self, d_qdesc, d_q, d_q_off, d_match, d_nmatches, d_claimed,
            stream=stream)

    def project_local_map(self, d_frames, d_mps, d_mp_off, max_mps: int, d_skip, d_q,
                          d_nvisible=None, th: float = 1.0, stream: int = 0):
        """SearchLocalPoints' projection loop for every frame (Tracking.cc:1322-1335): frame j's
        local MapPoints at [d_mp_off[j], d_mp_off[j+1]) of d_mps (MAP_POINT_DTYPE records),
        its pose in d_frames[j] (FRAME_POSE_DTYPE); isInFrustum(pMP, 0.5) writes the
        SearchByProjection query of each MapPoint into d_q (radius -1: not in view or d_skip
        set, i.e. bad or already matched), nToMatch into d_nvisible[j]."""
        is_in_frustum_batch_device(d_frames, self.batch, d_mps, d_mp_off, max_mps, d_skip, d_q,
                                   d_nvisible, 0.5, th, stream)

    def __call__(self, images, d_qdesc, d_q, d_q_off, d_match, d_nmatches, d_claimed=None,
                 stream: int = 0, local_map=None):
        """One tracking step of the B frames.  With `local_map` = (d_frames, d_mps, max_mps,
        d_skip, d_nvisible, th) the queries d_q are first projected from the local map
        (project_local_map, MapPoints indexed like the queries: d_q_off); without it d_q
        holds the caller's projections."""
        self.frames(images, stream)
        if local_map is not None:
            d_frames, d_mps, max_mps, d_skip, d_nvis, th = local_map
            self.project_local_map(d_frames, d_mps, d_q_off, max_mps, d_skip, d_q, d_nvis, th,
                                   stream)
        self.search_local_points(d_qdesc, d_q, d_q_off, d_match, d_nmatches, d_claimed, stream)

    def fetch_undistorted(self):
        """Host copies (nkp [B], undistorted keypoints [B, kp_cap], descriptors
        [B, kp_cap, 32]) of the last ``frames`` call."""
        import torch
        torch.cuda.synchronize(self.dev)
        nkp, _, desc = self.ext.batch_fetch(0, self.batch)
        ku = self.keys_un.cpu().numpy().view(KEYPOINT_DTYPE).reshape(self.batch, self.kp_cap)
        return nkp, ku, desc
