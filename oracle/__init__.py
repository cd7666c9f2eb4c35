"""ctypes front-end of the CPU restatement (oracle/_build/liborb_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker / the timed CPU baseline.  The product package
(my_orb_slam2_amd) never imports this module.

Parity status: the restatement follows the reference line by line (see orb_oracle.h for
file:line citations).  Its OpenCV 3.2 primitives (FAST, resize, GaussianBlur, fastAtan2)
are restated from OpenCV's published algorithm and are PARITY UNPINNED against the real
library, which is absent from this image; glibc cosf/sinf are the real glibc.
"""
from __future__ import annotations

import ctypes
import os
import pathlib
import subprocess

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
LIB_V3 = HERE / "_build" / "liborb_oracle.so"
LIB_V4 = HERE / "_build" / "liborb_oracle_v4.so"
AVX512 = ("avx512f", "avx512bw", "avx512cd", "avx512dq", "avx512vl")


def host_has_v4() -> bool:
    """x86-64-v4 (AVX-512 F/BW/CD/DQ/VL) on this host's CPU."""
    try:
        flags = next(l for l in open("/proc/cpuinfo") if l.startswith("flags")).split()
    except (OSError, StopIteration):
        return False
    return all(f in flags for f in AVX512)


# the build a -march=native compile would come closest to on this host
LIB_PATH = LIB_V4 if LIB_V4.exists() and host_has_v4() else LIB_V3
ISA = "x86-64-v4" if LIB_PATH == LIB_V4 else "x86-64-v3"

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

_lib = None


def build(force: bool = False) -> pathlib.Path:
    """Compile the restatement with its Makefile (g++; no GPU needed)."""
    srcs = list(HERE.glob("*.cpp")) + list(HERE.glob("*.h"))
    stale = any(not p.exists() for p in (LIB_V3, LIB_V4)) or \
        any(p.stat().st_mtime > min(LIB_V3.stat().st_mtime, LIB_V4.stat().st_mtime) for p in srcs)
    if force or stale:
        subprocess.run(["make", "-s", "-B" if force else "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        vp, i32, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.oracle_extractor_create.restype = vp
        L.oracle_extractor_create.argtypes = [i32, f32, i32, i32, i32, i32]
        L.oracle_extractor_destroy.argtypes = [vp]
        L.oracle_extract.argtypes = [vp, vp, i32, i32, i32]
        L.oracle_num_keypoints.argtypes = [vp]
        L.oracle_get_keypoints.argtypes = [vp, vp, i32]
        L.oracle_get_descriptors.argtypes = [vp, vp, i32]
        L.oracle_num_levels.argtypes = [vp]
        L.oracle_level_size.argtypes = [vp, i32, vp, vp]
        L.oracle_get_level.argtypes = [vp, i32, i32, vp]
        L.oracle_get_candidates.argtypes = [vp, i32, vp, i32]
        L.oracle_get_level_keypoints.argtypes = [vp, i32, vp, i32]
        L.oracle_get_tables.argtypes = [vp] * 7
        L.oracle_stereo_match.argtypes = [vp, vp, f32, f32, vp, vp]
        L.oracle_resize.argtypes = [vp, i32, i32, i32, vp, i32, i32, i32]
        L.oracle_gaussian7.argtypes = [vp, i32, i32, i32, vp, i32]
        L.oracle_fast.argtypes = [vp, i32, i32, i32, i32, vp, i32]
        L.oracle_fast_atan2.restype = f32
        L.oracle_fast_atan2.argtypes = [f32, f32]
        L.oracle_gaussian_taps.argtypes = [vp]
        L.oracle_descriptor_distance.argtypes = [vp, vp]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleExtractor:
    """Mirror of ORB_SLAM2::ORBextractor (src/ORBextractor.cc) on the CPU restatement."""

    def __init__(self, nfeatures=2000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7,
                 simd=1):
        self.nlevels = nlevels
        self._h = lib().oracle_extractor_create(nfeatures, scaleFactor, nlevels, iniThFAST,
                                                minThFAST, simd)

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.oracle_extractor_destroy(self._h)
            self._h = None

    def __call__(self, image: np.ndarray):
        img = np.ascontiguousarray(image, dtype=np.uint8)
        n = lib().oracle_extract(self._h, _p(img), img.shape[1], img.shape[0], img.shape[1])
        if n < 0:
            return None, None
        kps = np.zeros(n, KEYPOINT_DTYPE)
        desc = np.zeros((n, 32), np.uint8)
        lib().oracle_get_keypoints(self._h, _p(kps), n)
        lib().oracle_get_descriptors(self._h, _p(desc), n)
        return kps, (desc if n > 0 else None)   # the reference releases an empty Mat

    def level_size(self, level):
        w, h = ctypes.c_int(), ctypes.c_int()
        lib().oracle_level_size(self._h, level, ctypes.byref(w), ctypes.byref(h))
        return w.value, h.value

    def level(self, level, blurred=False):
        w, h = self.level_size(level)
        out = np.zeros((h, w), np.uint8)
        n = lib().oracle_get_level(self._h, level, 1 if blurred else 0, _p(out))
        return out if n > 0 else None

    def candidates(self, level):
        n = lib().oracle_get_candidates(self._h, level, None, 0)
        out = np.zeros(n, KEYPOINT_DTYPE)
        lib().oracle_get_candidates(self._h, level, _p(out), n)
        return out

    def level_keypoints(self, level):
        n = lib().oracle_get_level_keypoints(self._h, level, None, 0)
        out = np.zeros(n, KEYPOINT_DTYPE)
        lib().oracle_get_level_keypoints(self._h, level, _p(out), n)
        return out

    def tables(self):
        L = self.nlevels
        f = [np.zeros(L, np.float32) for _ in range(4)]
        feats = np.zeros(L, np.int32)
        umax = np.zeros(16, np.int32)
        lib().oracle_get_tables(self._h, *[_p(a) for a in f], _p(feats), _p(umax))
        return dict(scale=f[0], inv_scale=f[1], sigma2=f[2], inv_sigma2=f[3],
                    features_per_level=feats, umax=umax)


def stereo_match(left: OracleExtractor, right: OracleExtractor, n_left: int, mbf: float,
                 mb: float):
    """Frame::ComputeStereoMatches (src/Frame.cc:496-686) over the two last extractions."""
    u = np.zeros(n_left, np.float32)
    d = np.zeros(n_left, np.float32)
    nvalid = lib().oracle_stereo_match(left._h, right._h, mbf, mb, _p(u), _p(d))
    return u, d, nvalid


def resize(src: np.ndarray, dw: int, dh: int, simd: int = 1) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros((dh, dw), np.uint8)
    lib().oracle_resize(_p(src), src.shape[1], src.shape[0], src.shape[1], _p(dst), dw, dh, simd)
    return dst


def gaussian7(src: np.ndarray, simd: int = 1) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros_like(src)
    lib().oracle_gaussian7(_p(src), src.shape[1], src.shape[0], src.shape[1], _p(dst), simd)
    return dst


def fast(img: np.ndarray, threshold: int) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    n = lib().oracle_fast(_p(img), img.shape[1], img.shape[0], img.shape[1], threshold, None, 0)
    out = np.zeros(n, KEYPOINT_DTYPE)
    lib().oracle_fast(_p(img), img.shape[1], img.shape[0], img.shape[1], threshold, _p(out), n)
    return out


def fast_atan2(y: float, x: float) -> float:
    return lib().oracle_fast_atan2(y, x)


def gaussian_taps():
    t = np.zeros(7, np.int32)
    lib().oracle_gaussian_taps(_p(t))
    return t


def descriptor_distance(a, b):
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().oracle_descriptor_distance(_p(a), _p(b))
