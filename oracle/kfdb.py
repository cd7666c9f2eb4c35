"""ctypes front-end of the KeyFrameDatabase restatement (oracle/orb_kfdb_oracle.cpp).

TEST INFRASTRUCTURE ONLY: the checker of my_orb_slam2_amd.kfdb (same API, slots = add
order).  Parity status: restated statement by statement from src/KeyFrameDatabase.cc; the
reference itself cannot be built here (OpenCV / DBoW2 objects), so this is pinned only by the
cross-check against the pure-Python restatement in tests/test_kfdb.py.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import lib

_vp, _i = ctypes.c_void_p, ctypes.c_int


def _a(x):
    return x.ctypes.data_as(ctypes.c_void_p)


def _setup(L):
    if getattr(L, "_kfdb_ready", False):
        return L
    L.oracle_kfdb_create.restype = _vp
    L.oracle_kfdb_create.argtypes = [_i]
    L.oracle_kfdb_destroy.argtypes = [_vp]
    L.oracle_kfdb_add.restype = _i
    L.oracle_kfdb_add.argtypes = [_vp, _vp, _vp, _i]
    L.oracle_kfdb_erase.argtypes = [_vp, _i]
    L.oracle_kfdb_clear.argtypes = [_vp]
    L.oracle_kfdb_set_covisibles.argtypes = [_vp, _i, _vp, _i]
    L.oracle_kfdb_detect_reloc.restype = _i
    L.oracle_kfdb_detect_reloc.argtypes = [_vp, _vp, _vp, _i, _vp, _i]
    L.oracle_kfdb_detect_loop.restype = _i
    L.oracle_kfdb_detect_loop.argtypes = [_vp, _vp, _vp, _i, _vp, _i, ctypes.c_float, _vp, _i]
    L._kfdb_ready = True
    return L


class OracleKeyFrameDatabase:
    def __init__(self, covisibles: int = 10):
        self._L = _setup(lib())
        self._h = self._L.oracle_kfdb_create(covisibles)
        self.n = 0

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.oracle_kfdb_destroy(self._h)
            self._h = None

    def add(self, bow) -> int:
        w = np.ascontiguousarray(bow[0], np.uint32)
        v = np.ascontiguousarray(bow[1], np.float64)
        self.n += 1
        return self._L.oracle_kfdb_add(self._h, _a(w), _a(v), len(w))

    def erase(self, slot):
        self._L.oracle_kfdb_erase(self._h, int(slot))

    def clear(self):
        self._L.oracle_kfdb_clear(self._h)
        self.n = 0

    def set_covisibles(self, slot, neighbours):
        nb = np.ascontiguousarray(neighbours, np.int32)
        self._L.oracle_kfdb_set_covisibles(self._h, int(slot), _a(nb), len(nb))

    def DetectRelocalizationCandidates(self, bow):
        w = np.ascontiguousarray(bow[0], np.uint32)
        v = np.ascontiguousarray(bow[1], np.float64)
        out = np.zeros(max(self.n, 1), np.int32)
        k = self._L.oracle_kfdb_detect_reloc(self._h, _a(w), _a(v), len(w), _a(out), len(out))
        return out[:k].copy()

    def DetectLoopCandidates(self, bow, connected, minScore):
        w = np.ascontiguousarray(bow[0], np.uint32)
        v = np.ascontiguousarray(bow[1], np.float64)
        c = np.ascontiguousarray(connected, np.int32)
        out = np.zeros(max(self.n, 1), np.int32)
        k = self._L.oracle_kfdb_detect_loop(self._h, _a(w), _a(v), len(w), _a(c), len(c),
                                            float(minScore), _a(out), len(out))
        return out[:k].copy()
