"""KeyFrameDatabase over liborbx.so (include/orbx_kfdb.h).

Mirrors ORB_SLAM2::KeyFrameDatabase (include/KeyFrameDatabase.h:40-66,
src/KeyFrameDatabase.cc): ``add`` / ``erase`` / ``clear`` and the two candidate detectors.
Keyframes are the slots ``add`` returns (the caller keeps the KeyFrame* <-> slot map); a
BowVector is a ``(words, values)`` pair with word ids ascending (DBoW2::BowVector order).
The covisibility lists the detectors accumulate over (KeyFrame::GetBestCovisibilityKeyFrames)
are set per slot with ``set_covisibles`` whenever the Map updates them.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, load, ptr

ORBX_ERR_CAPACITY = -3


class KfdbParams(ctypes.Structure):
    _fields_ = [("covisibles", ctypes.c_int32), ("device", ctypes.c_int32)]


def _bow(bow):
    w = np.ascontiguousarray(bow[0], np.uint32)
    v = np.ascontiguousarray(bow[1], np.float64)
    if len(w) != len(v):
        raise ValueError("BowVector words and values differ in length")
    return w, v


class KeyFrameDatabase:
    def __init__(self, covisibles: int = 10, device: int = 0):
        self._L = load()
        self.params = KfdbParams(covisibles, device)
        h = ctypes.c_void_p()
        check("orbx_kfdb_create", self._L.orbx_kfdb_create(ctypes.byref(self.params),
                                                            ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.orbx_kfdb_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add(self, bow) -> int:
        """KeyFrameDatabase::add (:40-46); returns the keyframe's slot."""
        w, v = _bow(bow)
        slot = ctypes.c_int32(-1)
        check("orbx_kfdb_add", self._L.orbx_kfdb_add(self._h, ptr(w), ptr(v), len(w),
                                                      ctypes.byref(slot)))
        return slot.value

    def erase(self, slot: int):
        """KeyFrameDatabase::erase (:48-67)."""
        check("orbx_kfdb_erase", self._L.orbx_kfdb_erase(self._h, int(slot)))

    def clear(self):
        """KeyFrameDatabase::clear (:69-73)."""
        check("orbx_kfdb_clear", self._L.orbx_kfdb_clear(self._h))

    def __len__(self):
        n = ctypes.c_int32(0)
        check("orbx_kfdb_size", self._L.orbx_kfdb_size(self._h, ctypes.byref(n)))
        return n.value

    def set_covisibles(self, slot: int, neighbours):
        """The slot's mvpOrderedConnectedKeyFrames (weight-descending slots)."""
        nb = np.ascontiguousarray(neighbours, np.int32)
        check("orbx_kfdb_set_covisibles", self._L.orbx_kfdb_set_covisibles(
            self._h, int(slot), ptr(nb), len(nb)))

    def _result(self, fn, name, *args):
        """Runs a detector into a buffer sized from the database; if keyframes were added
        concurrently and the list outgrew it (ORBX_ERR_CAPACITY, *ncand = the true count), runs
        it again with room for that count."""
        cap = max(len(self), 1)
        for _ in range(4):
            out = np.zeros(cap, np.int32)
            n = ctypes.c_int32(0)
            code = fn(*args, ptr(out), cap, ctypes.byref(n))
            if code == ORBX_ERR_CAPACITY and n.value > cap:
                cap = max(n.value, len(self), 1)
                continue
            check(name, code)
            return out[:n.value].copy()
        check(name, code)

    def DetectRelocalizationCandidates(self, bow) -> np.ndarray:
        """KeyFrameDatabase::DetectRelocalizationCandidates (:220-337): candidate slots."""
        w, v = _bow(bow)
        return self._result(self._L.orbx_kfdb_detect_relocalization,
                            "orbx_kfdb_detect_relocalization", self._h, ptr(w), ptr(v), len(w))

    def DetectLoopCandidates(self, bow, connected, minScore: float) -> np.ndarray:
        """KeyFrameDatabase::DetectLoopCandidates (:76-208); `connected` = the slots of the
        query keyframe's GetConnectedKeyFrames()."""
        w, v = _bow(bow)
        c = np.ascontiguousarray(connected, np.int32)
        return self._result(self._L.orbx_kfdb_detect_loop, "orbx_kfdb_detect_loop", self._h,
                            ptr(w), ptr(v), len(w), ptr(c), len(c), float(minScore))

    def last_timing(self):
        """(scan_ms, select_ms) of the last detect call (HIP events on the database stream)."""
        a, b = ctypes.c_double(), ctypes.c_double()
        check("orbx_kfdb_last_timing", self._L.orbx_kfdb_last_timing(self._h, ctypes.byref(a),
                                                                      ctypes.byref(b)))
        return a.value, b.value
