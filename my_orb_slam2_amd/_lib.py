"""ctypes binding of liborbx.so (include/orbx.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU is present,
constructing an extractor raises.  Loading the library itself needs no GPU (the CPU test
suite checks that every symbol of include/orbx.h is exported).
"""
from __future__ import annotations

import ctypes
import pathlib

import numpy as np

PKG = pathlib.Path(__file__).resolve().parent
LIB_PATH = PKG / "liborbx.so"
# tools/variants.py benchmarks alternative builds of the same sources (in-tree .so files)
ORBX_LIB_ENV = "ORBX_LIB"

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

KERNELS = ["k_level", "k_fast", "k_octree", "k_orient_desc", "k_stereo", "k_level0"]
MATCH_KERNELS = ["k_bow", "k_triangulate", "k_proj_search", "k_proj_resolve", "k_distinctive",
                 "k_bf"]

STATUS = {0: "ORBX_OK", -1: "ORBX_ERR_INVALID", -2: "ORBX_ERR_DEVICE", -3: "ORBX_ERR_CAPACITY",
          -4: "ORBX_ERR_UNSUPPORTED", -5: "ORBX_ERR_STATE"}


class OrbxError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__(f"{fn} failed: {STATUS.get(code, code)}")
        self.code = code


class ExtractorParams(ctypes.Structure):
    _fields_ = [("nfeatures", ctypes.c_int), ("scale_factor", ctypes.c_float),
                ("nlevels", ctypes.c_int), ("ini_th_fast", ctypes.c_int),
                ("min_th_fast", ctypes.c_int), ("cv_simd", ctypes.c_int),
                ("max_batch", ctypes.c_int), ("device", ctypes.c_int)]


class BatchView(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int), ("kp_cap", ctypes.c_int), ("kps", ctypes.c_void_p),
                ("desc", ctypes.c_void_p), ("nkp", ctypes.c_void_p),
                ("pyramid", ctypes.c_void_p), ("pyr_bytes", ctypes.c_size_t),
                ("level_w", ctypes.c_int * 16), ("level_h", ctypes.c_int * 16),
                ("level_pitch", ctypes.c_int * 16), ("level_off", ctypes.c_size_t * 16)]


# name -> (restype, argtypes); the exported C ABI (include/orbx.h)
_vp, _i, _f, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
SIGNATURES = {
    "orbx_extractor_create": (_i, [ctypes.POINTER(ExtractorParams), ctypes.POINTER(_vp)]),
    "orbx_extractor_destroy": (_i, [_vp]),
    "orbx_extractor_tables": (_i, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "orbx_extractor_prepare": (_i, [_vp, _i, _i, _i, ctypes.POINTER(_i)]),
    "orbx_extract": (_i, [_vp, _vp, _i, _i, _sz, _vp, _i, _vp, ctypes.POINTER(_i)]),
    "orbx_stereo_frame_view": (_i, [_vp, _vp, _sz, _vp, _sz, _i, _i, ctypes.c_float,
                                    ctypes.c_float, _vp]),
    "orbx_extract_view": (_i, [_vp, _vp, _i, _i, _sz, ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                               ctypes.POINTER(_i)]),
    "orbx_pyramid_level": (_i, [_vp, _i, _i, _vp, ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    "orbx_extractor_keep_pyramid": (_i, [_vp, _i]),
    "orbx_frame_server_get_stats": (_i, [_vp, _vp, _i]),
    "orbx_frame_server_release": (_i, [_vp]),
    "orbx_blur_level": (_i, [_vp, _i, _i, _vp, ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    "orbx_extract_batch_device": (_i, [_vp, _vp, _i, _i, _i, _sz, _sz, _vp]),
    "orbx_batch_view_get": (_i, [_vp, ctypes.POINTER(BatchView)]),
    "orbx_batch_input_view": (_i, [_vp, _i, _i, _i, ctypes.POINTER(_vp), ctypes.POINTER(_sz),
                                   ctypes.POINTER(_sz)]),
    "orbx_extract_batch_resident": (_i, [_vp, _i, _vp]),
    "orbx_stereo_frames_resident": (_i, [_vp, _i, _f, _f, _vp, _vp, _vp, _vp]),
    "orbx_batch_fetch": (_i, [_vp, _i, _i, _vp, _vp, _vp]),
    "orbx_stereo_match": (_i, [_vp, _vp, _f, _f, _vp, _vp, _i, ctypes.POINTER(_i)]),
    "orbx_stereo_match_batch_device": (_i, [_vp, _vp, _f, _f, _vp, _vp, _vp, _vp]),
    "orbx_stereo_frames_device": (_i, [_vp, _vp, _vp, _i, _i, _i, _sz, _sz, _f, _f, _vp, _vp,
                                       _vp, _vp]),
    "orbx_descriptor_distance": (_i, [_vp, _vp]),
    "orbx_version": (ctypes.c_char_p, []),
    "orbx_last_error": (ctypes.c_char_p, []),
    "orbx_device_count": (_i, [ctypes.POINTER(_i)]),
    "orbx_extractor_set_overlap": (_i, [_vp, _i, _i, _i]),
    "orbx_extractor_get_overlap": (_i, [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i),
                                        ctypes.POINTER(_i)]),
    "orbx_profile_enable": (_i, [_vp, _i]),
    "orbx_profile_collect": (_i, [_vp, _vp, _vp]),
    "orbx_kernel_name": (ctypes.c_char_p, [_i]),
    "orbx_extractor_launch_info": (_i, [_vp, _i, _vp, ctypes.POINTER(_i)]),
    # include/orbx_match.h
    "orbx_matcher_create": (_i, [_vp, ctypes.POINTER(_vp)]),
    "orbx_matcher_destroy": (_i, [_vp]),
    "orbx_compute_three_maxima": (None, [_vp, _i, _vp, _vp, _vp]),
    "orbx_search_by_bow_kf_frame": (_i, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "orbx_search_by_bow_kf_kf": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "orbx_search_for_triangulation": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _f, _f, _vp, _vp, _i,
                                           _i, _vp, _i, _vp]),
    "orbx_search_by_projection": (_i, [_vp, _i, _vp, _vp, _vp, _vp, _i, _vp, _i, _i, _vp, _vp]),
    "orbx_search_by_projection_ex": (_i, [_vp, _i, _vp, _vp, _vp, _vp, _vp, _i, _vp, _i, _i, _i,
                                          _vp, _vp]),
    "orbx_search_by_sim3": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _i, _vp, _vp]),
    "orbx_search_for_initialization": (_i, [_vp, _vp, _vp, _vp, _i, _vp, _vp]),
    "orbx_search_by_bow_kf_frame_batch_device": (_i, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "orbx_search_for_triangulation_batch_device": (_i, [_vp, _vp, _i, _vp, _vp, _vp, _vp, _vp,
                                                        _vp, _i, _i, _vp, _vp, _vp, _vp]),
    "orbx_search_by_projection_batch_device": (_i, [_vp, _i, _vp, _i, _vp, _vp, _i, _vp, _vp,
                                                    _vp, _vp, _i, _vp, _i, _i, _vp, _vp, _vp]),
    "orbx_matcher_sync": (_i, [_vp, _vp]),
    "orbx_kf_db_node_order": (_i, [_vp, _vp, _i, _vp, _vp, _vp, _vp, _vp]),
    "orbx_compute_distinctive_descriptors": (_i, [_vp, _vp, _vp, _i, _vp]),
    "orbx_compute_distinctive_descriptors_device": (_i, [_vp, _vp, _vp, _i, _vp, _vp]),
    "orbx_hamming_bf_top2": (_i, [_vp, _vp, _i, _vp, ctypes.c_int64, _vp, _vp, _vp]),
    "orbx_bf_kernel": (ctypes.c_char_p, []),
    "orbx_bf_kernel_name": (ctypes.c_char_p, [_i]),
    "orbx_matcher_set_bf_kernel": (_i, [_vp, _i]),
    "orbx_hamming_bf_top2_device": (_i, [_vp, _vp, _i, _vp, ctypes.c_int64, ctypes.c_int64,
                                         _vp, _vp, _vp, _vp]),
    "orbx_matcher_profile_enable": (_i, [_vp, _i]),
    "orbx_matcher_profile_collect": (_i, [_vp, _vp, _vp]),
    "orbx_match_kernel_name": (ctypes.c_char_p, [_i]),
    # include/orbx_vocab.h
    "orbx_vocabulary_load_text": (_i, [ctypes.c_char_p, _i, ctypes.POINTER(_vp)]),
    "orbx_vocabulary_destroy": (_i, [_vp]),
    "orbx_vocabulary_info": (_i, [_vp] + [_vp] * 6),
    "orbx_vocabulary_transform": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                       _vp]),
    "orbx_vocabulary_transform_device": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp]),
    "orbx_bow_score_l1": (ctypes.c_double, [_vp, _vp, _i, _vp, _vp, _i]),
    "orbx_bow_db_score": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _i]),
    "orbx_bow_db_score_device": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
    # include/orbx_kfdb.h
    "orbx_kfdb_create": (_i, [_vp, ctypes.POINTER(_vp)]),
    "orbx_kfdb_destroy": (_i, [_vp]),
    "orbx_kfdb_add": (_i, [_vp, _vp, _vp, _i, ctypes.POINTER(_i)]),
    "orbx_kfdb_erase": (_i, [_vp, _i]),
    "orbx_kfdb_clear": (_i, [_vp]),
    "orbx_kfdb_size": (_i, [_vp, ctypes.POINTER(_i)]),
    "orbx_kfdb_set_covisibles": (_i, [_vp, _i, _vp, _i]),
    "orbx_kfdb_detect_relocalization": (_i, [_vp, _vp, _vp, _i, _vp, _i, ctypes.POINTER(_i)]),
    "orbx_kfdb_detect_loop": (_i, [_vp, _vp, _vp, _i, _vp, _i, _f, _vp, _i, ctypes.POINTER(_i)]),
    "orbx_kfdb_last_timing": (_i, [_vp, ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_double)]),
    # include/orbx_frame.h
    "orbx_undistort_keypoints": (_i, [_vp, _vp, _i, _vp, _i, _vp, _i]),
    "orbx_undistort_keypoints_device": (_i, [_vp, _vp, _i, _vp, _i, _vp, _vp]),
    "orbx_image_bounds": (_i, [_vp, _vp, _i, _i, _i, _vp]),
    "orbx_assign_grid_device": (_i, [_vp, _i, _i, _i, _f, _f, _f, _f, _vp, _vp, _vp]),
    "orbx_assign_grid_batch_device": (_i, [_vp, _i, _vp, _i, _i, _i, _f, _f, _f, _f, _vp, _vp,
                                           _vp]),
    "orbx_undistort_keypoints_batch_device": (_i, [_vp, _vp, _i, _vp, _i, _vp, _i, _vp, _vp]),
    "orbx_cvt_color": (_i, [_vp, _i, _i, _sz, _i, _i, _vp, _sz, _i]),
    "orbx_cvt_color_device": (_i, [_vp, _i, _i, _sz, _i, _i, _vp, _sz, _vp]),
    "orbx_is_in_frustum_batch_device": (_i, [_vp, _i, _vp, _vp, _i, _vp, _f, _f, _vp, _vp, _vp]),
    "orbx_is_in_frustum": (_i, [_vp, _vp, _i, _vp, _f, _f, _vp, _vp, _i]),
}

_lib = None


def load(path: pathlib.Path | str | None = None):
    """Load liborbx.so (raises OSError if it has not been built)."""
    global _lib
    if _lib is None or path is not None:
        import os
        p = pathlib.Path(path or os.environ.get(ORBX_LIB_ENV) or LIB_PATH)
        # One HIP runtime per process: torch wheels bundle their own libamdhip64 (same
        # soname).  Loading torch first makes liborbx bind to that copy instead of pulling
        # in /opt/rocm's second runtime next to it.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not p.exists():
            raise OSError(f"{p} not found: build it with `python -m my_orb_slam2_amd.build`")
        L = ctypes.CDLL(str(p))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        if path is not None:
            return L
        _lib = L
    return _lib


def check(fn: str, code: int):
    if code != 0:
        err = OrbxError(fn, code)
        try:
            detail = load().orbx_last_error()
            if detail:
                err.args = (err.args[0] + " [" + detail.decode() + "]",)
        except Exception:
            pass
        raise err
    return code


def ptr(a) -> ctypes.c_void_p:
    """Address of a numpy array or a torch tensor (device or host)."""
    if isinstance(a, np.ndarray):
        return ctypes.c_void_p(a.ctypes.data)
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    if a is None:
        return ctypes.c_void_p(0)
    return ctypes.c_void_p(int(a))
