"""ORBextractor / stereo front-end over liborbx.so.

Mirrors the reference's operator interface:
  ORB_SLAM2::ORBextractor (include/ORBextractor.h:45-111, src/ORBextractor.cc:410-1154)
  Frame::ComputeStereoMatches (src/Frame.cc:496-686)
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import BatchView, ExtractorParams, KERNELS, KEYPOINT_DTYPE, check, load, ptr


class _DeviceArray:
    """A device uint8 array by address (__cuda_array_interface__, which torch.as_tensor wraps
    without copying)."""

    def __init__(self, ptr_value: int, shape, strides):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": "|u1",
                                         "data": (int(ptr_value), False),
                                         "strides": tuple(strides), "version": 2}


class ORBextractor:
    """ORB_SLAM2::ORBextractor on the GPU.

    ``extractor(image, mask)`` returns ``(keypoints, descriptors)`` like the reference's
    ``operator()(image, mask, keypoints, descriptors)``: keypoints as a structured array with
    cv::KeyPoint fields, descriptors as an (N, 32) uint8 array (None when N == 0, as the
    reference releases the Mat).  An empty image returns ``(None, None)`` (the reference
    returns without touching its outputs).  The mask is ignored, as in the reference.
    """

    def __init__(self, nfeatures: int = 1000, scaleFactor: float = 1.2, nlevels: int = 8,
                 iniThFAST: int = 20, minThFAST: int = 7, *, cv_simd: int = 1,
                 max_batch: int = 1, device: int = 0):
        self._L = load()
        self.params = ExtractorParams(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST,
                                      cv_simd, max_batch, device)
        h = ctypes.c_void_p()
        check("orbx_extractor_create",
              self._L.orbx_extractor_create(ctypes.byref(self.params), ctypes.byref(h)))
        self._h = h
        self.nlevels = nlevels
        n = nlevels
        self._tab = [np.zeros(n, np.float32) for _ in range(4)] + [np.zeros(n, np.int32)]
        check("orbx_extractor_tables", self._L.orbx_extractor_tables(self._h, *map(ptr, self._tab)))
        self._last_size = None
        self._nkp = 0

    def close(self):
        if getattr(self, "_h", None):
            self._L.orbx_extractor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- getters of include/ORBextractor.h:63-83 ----
    def GetLevels(self):
        return self.nlevels

    def GetScaleFactor(self):
        return float(self.params.scale_factor)

    def GetScaleFactors(self):
        return self._tab[0].copy()

    def GetInverseScaleFactors(self):
        return self._tab[1].copy()

    def GetScaleSigmaSquares(self):
        return self._tab[2].copy()

    def GetInverseScaleSigmaSquares(self):
        return self._tab[3].copy()

    @property
    def features_per_level(self):
        return self._tab[4].copy()

    # ---- operator() ----
    def __call__(self, image: np.ndarray, mask=None):
        img = np.ascontiguousarray(image, dtype=np.uint8)
        if img.size == 0:
            return None, None
        if img.ndim != 2:
            raise ValueError("ORBextractor expects a single-channel 8-bit image (CV_8UC1)")
        h, w = img.shape
        n = ctypes.c_int(0)
        cap = 1
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        code = self._L.orbx_extract(self._h, ptr(img), w, h, w, ptr(kps), cap, ptr(desc),
                                    ctypes.byref(n))
        if code == -3 or n.value > cap:   # capacity: fetch with the exact size
            cap = n.value
            kps = np.zeros(cap, KEYPOINT_DTYPE)
            desc = np.zeros((cap, 32), np.uint8)
            code = self._L.orbx_extract(self._h, ptr(img), w, h, w, ptr(kps), cap, ptr(desc),
                                        ctypes.byref(n))
        check("orbx_extract", code)
        self._last_size = (w, h)
        self._nkp = n.value
        kps = kps[: n.value]
        return kps, (desc[: n.value] if n.value > 0 else None)

    @property
    def mvImagePyramid(self):
        """Pyramid of the last call (include/ORBextractor.h:85), copied to host."""
        return [self.pyramid_level(l) for l in range(self.nlevels)]

    def pyramid_level(self, level: int, index: int = 0) -> np.ndarray:
        w, h = ctypes.c_int(), ctypes.c_int()
        check("orbx_pyramid_level", self._L.orbx_pyramid_level(
            self._h, index, level, None, ctypes.byref(w), ctypes.byref(h)))
        out = np.zeros((h.value, w.value), np.uint8)
        check("orbx_pyramid_level", self._L.orbx_pyramid_level(
            self._h, index, level, ptr(out), ctypes.byref(w), ctypes.byref(h)))
        return out

    def blur_level(self, level: int, index: int = 0) -> np.ndarray:
        """The 7x7 Gaussian of a level that the descriptors sample (ORBextractor.cc:1107-1108)."""
        w, h = ctypes.c_int(), ctypes.c_int()
        check("orbx_blur_level", self._L.orbx_blur_level(
            self._h, index, level, None, ctypes.byref(w), ctypes.byref(h)))
        out = np.zeros((h.value, w.value), np.uint8)
        check("orbx_blur_level", self._L.orbx_blur_level(
            self._h, index, level, ptr(out), ctypes.byref(w), ctypes.byref(h)))
        return out

    def keep_pyramid(self, on: bool = True):
        """orbx_extractor_keep_pyramid: after ``extract_stereo`` the handle holds both views'
        pyramids (image 0 = left, 1 = right) whether the frame ran alone or in a frame-server
        batch; off (the default) none in either case."""
        check("orbx_extractor_keep_pyramid", self._L.orbx_extractor_keep_pyramid(self._h, int(on)))

    def frame_server_stats(self, reset: bool = False) -> dict:
        """Counters of the frame server this handle's ``extract_stereo`` calls go to
        (orbx_frame_server_get_stats)."""
        st = FrameServerStats()
        check("orbx_frame_server_get_stats", self._L.orbx_frame_server_get_stats(
            self._h, ctypes.byref(st), int(reset)))
        return {"solo_calls": st.solo_calls, "batches": st.batches,
                "served_frames": st.served_frames,
                "batches_of_size": list(st.batches_of_size),
                "batches_per_pair": list(st.batches_per_pair),
                "peak_inflight": st.peak_inflight, "users": st.users,
                "resident": bool(st.resident)}

    def frame_server_release(self):
        """orbx_frame_server_release: free the frame server's resources now."""
        check("orbx_frame_server_release", self._L.orbx_frame_server_release(self._h))

    # ---- batched device path ----
    def prepare(self, width: int, height: int, batch: int) -> int:
        """Allocate the workspace for `batch` images of width x height; returns kp_cap."""
        kc = ctypes.c_int(0)
        check("orbx_extractor_prepare", self._L.orbx_extractor_prepare(
            self._h, width, height, batch, ctypes.byref(kc)))
        return kc.value

    def extract_batch_device(self, images, stream=None):
        """Extract a [B, H, W] uint8 CUDA/HIP tensor already resident in HBM."""
        B, H, W = images.shape
        stride = images.stride(1) * images.element_size()
        bstride = images.stride(0) * images.element_size()
        check("orbx_extract_batch_device", self._L.orbx_extract_batch_device(
            self._h, ptr(images), B, W, H, stride, bstride, ptr(stream)))

    def set_overlap(self, mode: int, fork_level: int = 3, levels: int = 1):
        """Side branch of the extraction (orbx_extractor_set_overlap): mode 0 = every kernel
        in sequence, 1-3 = the first `levels` levels' FAST (+ octree, + orientation) beside
        the pyramid chain, forked before level `fork_level`; mode < 0 = the built-in default."""
        check("orbx_extractor_set_overlap",
              self._L.orbx_extractor_set_overlap(self._h, mode, fork_level, levels))

    def overlap(self):
        """(mode, fork_level, levels) of the side branch."""
        m, f, l = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check("orbx_extractor_get_overlap", self._L.orbx_extractor_get_overlap(
            self._h, ctypes.byref(m), ctypes.byref(f), ctypes.byref(l)))
        return m.value, f.value, l.value

    def profile(self, on: bool = True):
        """Bracket every kernel launch with HIP events (on its launch stream)."""
        check("orbx_profile_enable", self._L.orbx_profile_enable(self._h, 1 if on else 0))

    def collect_profile(self) -> dict:
        """{kernel: (total_ms, launches)} since the last collect (waits for the launches)."""
        ms = np.zeros(len(KERNELS), np.float64)
        n = np.zeros(len(KERNELS), np.int64)
        check("orbx_profile_collect", self._L.orbx_profile_collect(self._h, ptr(ms), ptr(n)))
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(KERNELS)}

    def batch_fetch(self, first: int = 0, count: int | None = None):
        """Host copies (nkp, keypoints, descriptors) of images [first, first+count) of the last
        batched call; keypoints/descriptors are [count, kp_cap] arrays (rows >= nkp unused)."""
        v = self.batch_view()
        count = v.batch - first if count is None else count
        nkp = np.zeros(count, np.int32)
        kps = np.zeros((count, v.kp_cap), KEYPOINT_DTYPE)
        desc = np.zeros((count, v.kp_cap, 32), np.uint8)
        check("orbx_batch_fetch", self._L.orbx_batch_fetch(self._h, first, count, ptr(nkp),
                                                            ptr(kps), ptr(desc)))
        return nkp, kps, desc

    def input_views(self, width: int, height: int, batch: int):
        """The pyramid's level-0 slots of `batch` images as a [batch, height, width] uint8
        torch tensor on the device (a view, no copy; include/orbx.h orbx_batch_input_view):
        images written there are extracted by ``extract_batch_resident`` without the input
        copy.  Valid until a call with another size or a larger batch."""
        import torch
        p, pitch, istride = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_size_t()
        check("orbx_batch_input_view", self._L.orbx_batch_input_view(
            self._h, width, height, batch, ctypes.byref(p), ctypes.byref(pitch),
            ctypes.byref(istride)))
        return torch.as_tensor(_DeviceArray(p.value, (batch, height, width),
                                            (istride.value, pitch.value, 1)),
                               device=torch.device("cuda", self.params.device))

    def extract_batch_resident(self, batch: int, stream=None):
        """Extract the `batch` images already in the level-0 slots (``input_views``)."""
        check("orbx_extract_batch_resident", self._L.orbx_extract_batch_resident(
            self._h, batch, ptr(stream)))

    def launch_info(self, batch: int):
        """(strip rows per level, stereo workgroups per pair) of a batched call of `batch`
        images at the prepared size (include/orbx.h orbx_extractor_launch_info)."""
        rows = np.zeros(self.nlevels, np.int32)
        split = ctypes.c_int(0)
        check("orbx_extractor_launch_info", self._L.orbx_extractor_launch_info(
            self._h, batch, ptr(rows), ctypes.byref(split)))
        return rows, split.value

    def batch_view(self) -> BatchView:
        v = BatchView()
        check("orbx_batch_view_get", self._L.orbx_batch_view_get(self._h, ctypes.byref(v)))
        return v


def compute_stereo_matches(left: ORBextractor, right: ORBextractor, mbf: float, mb: float):
    """Frame::ComputeStereoMatches over the last extraction of `left` and `right`.

    Returns (mvuRight, mvDepth, n_valid); -1 marks a left keypoint without a match.  `mb` is
    the term the reference reads at src/Frame.cc:534 (normally mbf / fx).
    """
    n = left._nkp
    u = np.zeros(max(n, 1), np.float32)
    d = np.zeros(max(n, 1), np.float32)
    nv = ctypes.c_int(0)
    check("orbx_stereo_match", left._L.orbx_stereo_match(
        left._h, right._h, mbf, mb, ptr(u), ptr(d), n, ctypes.byref(nv)))
    return u[:n], d[:n], nv.value


class FrameServerStats(ctypes.Structure):
    """orbx_frame_server_stats (include/orbx.h)."""
    _fields_ = [("solo_calls", ctypes.c_int64), ("batches", ctypes.c_int64),
                ("served_frames", ctypes.c_int64), ("batches_of_size", ctypes.c_int64 * 9),
                ("batches_per_pair", ctypes.c_int64 * 2), ("peak_inflight", ctypes.c_int32),
                ("users", ctypes.c_int32), ("resident", ctypes.c_int32)]


class StereoFrameOut(ctypes.Structure):
    """orbx_stereo_frame_out (include/orbx.h)."""
    _fields_ = [("kps", ctypes.c_void_p * 2), ("desc", ctypes.c_void_p * 2),
                ("n", ctypes.c_int32 * 2), ("u_right", ctypes.c_void_p),
                ("depth", ctypes.c_void_p), ("n_valid", ctypes.c_int32)]


def extract_stereo(ext: ORBextractor, left: np.ndarray, right: np.ndarray, mbf: float,
                   mb: float):
    """The stereo Frame constructor's extraction and matching (src/Frame.cc:89-102) as one
    call on one extractor (orbx_stereo_frame_view: both views as a two-image batch with the
    stereo match appended, one graph replay, one wait).  Returns (kps_left, desc_left,
    kps_right, desc_right, mvuRight, mvDepth, n_valid), equal to two extractions +
    ``compute_stereo_matches``."""
    L = np.ascontiguousarray(left, dtype=np.uint8)
    R = np.ascontiguousarray(right, dtype=np.uint8)
    if L.ndim != 2 or L.shape != R.shape:
        raise ValueError("extract_stereo expects two single-channel images of one size")
    h, w = L.shape
    o = StereoFrameOut()
    check("orbx_stereo_frame_view", ext._L.orbx_stereo_frame_view(
        ext._h, ptr(L), w, ptr(R), w, w, h, mbf, mb, ctypes.byref(o)))

    def arr(addr, n, dtype, shape):
        if n <= 0:
            return np.zeros(shape, dtype)
        buf = (ctypes.c_uint8 * (n * np.dtype(dtype).itemsize * int(np.prod(shape[1:]) or 1)))
        return np.frombuffer(buf.from_address(addr), dtype).reshape(shape).copy()

    nl, nr = o.n[0], o.n[1]
    kl = arr(o.kps[0], nl, KEYPOINT_DTYPE, (nl,))
    kr = arr(o.kps[1], nr, KEYPOINT_DTYPE, (nr,))
    dl = arr(o.desc[0], nl, np.uint8, (nl, 32))
    dr = arr(o.desc[1], nr, np.uint8, (nr, 32))
    u = arr(o.u_right, nl, np.float32, (nl,))
    d = arr(o.depth, nl, np.float32, (nl,))
    ext._nkp = -1   # the handle now holds a two-image batch, not a single-image extraction
    return kl, dl, kr, dr, u, d, o.n_valid


class StereoBatch:
    """Batched stereo front-end: B rectified pairs per call, all on one HIP stream.

    The reference's stereo Frame runs two ORBextractor objects with the same parameters on
    the left and right images (src/Frame.cc:89-92, Tracking.cc:136-139) and then
    ComputeStereoMatches (:102).  Here one handle extracts the 2B views as one batch
    (images [0,B) left, [B,2B) right) and matches image i with image B+i.  Outputs stay in
    HBM; ``fetch`` copies them to host.
    """

    def __init__(self, batch: int, nfeatures=2000, scaleFactor=1.2, nlevels=8, iniThFAST=20,
                 minThFAST=7, cv_simd=1, device=0):
        import torch
        self.batch = batch
        self.ext = ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST,
                                cv_simd=cv_simd, max_batch=2 * batch, device=device)
        self.device = torch.device("cuda", device)
        self.uR = self.depth = self.nvalid = None
        self._alloc_key = None    # (B, W, H, kp_cap) of the output buffers
        self._last_b = None       # B of the last call: the right views start at image B

    def __call__(self, left_imgs, right_imgs, mbf: float, mb: float, stream=None):
        import torch
        B, H, W = left_imgs.shape
        assert right_imgs.shape == left_imgs.shape
        assert left_imgs.stride() == right_imgs.stride(), "left/right tensors need equal strides"
        st = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        if self._alloc_key is None or self._alloc_key[:3] != (B, W, H):
            # kp_cap follows W and H (the octree root count), so any shape change
            # reallocates: k_stereo writes rows of kp_cap floats per pair
            kc = self.ext.prepare(W, H, 2 * B)
            if self._alloc_key is None or self._alloc_key[0] != B or self._alloc_key[3] != kc:
                self.uR = torch.empty((B, kc), dtype=torch.float32, device=self.device)
                self.depth = torch.empty((B, kc), dtype=torch.float32, device=self.device)
                self.nvalid = torch.empty((B,), dtype=torch.int32, device=self.device)
            self._alloc_key = (B, W, H, kc)
        stride = left_imgs.stride(1) * left_imgs.element_size()
        bstride = left_imgs.stride(0) * left_imgs.element_size()
        check("orbx_stereo_frames_device", self.ext._L.orbx_stereo_frames_device(
            self.ext._h, ptr(left_imgs), ptr(right_imgs), B, W, H, stride, bstride, mbf, mb,
            ptr(self.uR), ptr(self.depth), ptr(self.nvalid), ctypes.c_void_p(st)))
        self._last_b = B
        return self.uR, self.depth, self.nvalid

    def input_views(self, width: int, height: int):
        """(left, right) [B, H, W] device views of the pyramid's level-0 slots: pairs written
        there run through ``run_resident`` without the device copy of the input images."""
        v = self.ext.input_views(width, height, 2 * self.batch)
        self._prepare_outputs(width, height)
        return v[:self.batch], v[self.batch:]

    def _prepare_outputs(self, W, H):
        import torch
        B = self.batch
        if self._alloc_key is None or self._alloc_key[:3] != (B, W, H):
            kc = self.ext.prepare(W, H, 2 * B)
            if self._alloc_key is None or self._alloc_key[0] != B or self._alloc_key[3] != kc:
                self.uR = torch.empty((B, kc), dtype=torch.float32, device=self.device)
                self.depth = torch.empty((B, kc), dtype=torch.float32, device=self.device)
                self.nvalid = torch.empty((B,), dtype=torch.int32, device=self.device)
            self._alloc_key = (B, W, H, kc)

    def run_resident(self, mbf: float, mb: float, stream=None):
        """The stereo front-end over the B pairs in ``input_views`` (orbx_stereo_frames_resident)."""
        import torch
        if self._alloc_key is None:
            raise RuntimeError("run_resident before input_views")
        st = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        check("orbx_stereo_frames_resident", self.ext._L.orbx_stereo_frames_resident(
            self.ext._h, self.batch, mbf, mb, ptr(self.uR), ptr(self.depth), ptr(self.nvalid),
            ctypes.c_void_p(st)))
        self._last_b = self.batch
        return self.uR, self.depth, self.nvalid

    def fetch(self, side: str = "left"):
        """Host copies (nkp, keypoints, descriptors) of the left or right views of the last
        call (left view of pair i = image i, right view = image B + i)."""
        if self._last_b is None:
            raise RuntimeError("StereoBatch.fetch before any call")
        if side not in ("left", "right"):
            raise ValueError("side must be 'left' or 'right'")
        B = self._last_b
        return self.ext.batch_fetch(0 if side == "left" else B, B)

    def profile(self, on: bool = True):
        self.ext.profile(on)

    def collect_profile(self):
        return self.ext.collect_profile()
