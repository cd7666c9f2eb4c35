"""ORBVocabulary (DBoW2 TemplatedVocabulary<FORB>) over liborbx.so (include/orbx_vocab.h).

``Vocabulary.load_text`` replaces TemplatedVocabulary::loadFromTextFile
(Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1417); ``transform`` replaces
Frame::ComputeBoW's transform(desc, mBowVec, mFeatVec, 4) (src/Frame.cc:420-427) and returns
the BowVector and the FeatureVector the matchers take.  The descent runs on the GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, load, ptr
from .features import FeatureVector

_i32 = ctypes.c_int32


class Vocabulary:
    """ORB_SLAM2::ORBVocabulary loaded from the DBoW2 text format."""

    def __init__(self, handle, lib):
        self._h, self._L = handle, lib
        vals = [_i32() for _ in range(6)]
        check("orbx_vocabulary_info", lib.orbx_vocabulary_info(handle, *[ctypes.byref(v) for v in vals]))
        self.k, self.L, self.scoring, self.weighting, self.n_nodes, self.n_words = (
            v.value for v in vals)

    @classmethod
    def load_text(cls, path: str, device: int = 0) -> "Vocabulary":
        L = load()
        h = ctypes.c_void_p()
        check("orbx_vocabulary_load_text",
              L.orbx_vocabulary_load_text(str(path).encode(), device, ctypes.byref(h)))
        return cls(h, L)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._L.orbx_vocabulary_destroy(h)
            self._h = None

    def transform(self, desc, levelsup: int = 4):
        """-> (words, nodes, (bow_words, bow_values), FeatureVector)."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        cap = max(n, 1)
        word, node = np.zeros(cap, np.int32), np.zeros(cap, np.int32)
        bw, bv = np.zeros(cap, np.uint32), np.zeros(cap, np.float64)
        fn, fo, ff = np.zeros(cap, np.uint32), np.zeros(cap + 1, np.int32), np.zeros(cap, np.int32)
        nb, nf = _i32(), _i32()
        check("orbx_vocabulary_transform", self._L.orbx_vocabulary_transform(
            self._h, ptr(d), n, levelsup, ptr(word), ptr(node), ptr(bw), ptr(bv),
            ctypes.byref(nb), ptr(fn), ptr(fo), ptr(ff), ctypes.byref(nf)))
        fv = FeatureVector(fn[:nf.value].copy(), fo[:nf.value + 1].copy(),
                           ff[:fo[nf.value]].copy())
        return word[:n], node[:n], (bw[:nb.value].copy(), bv[:nb.value].copy()), fv


def bow_score_l1(bow1, bow2) -> float:
    """L1Scoring::score (Thirdparty/DBoW2/DBoW2/ScoringObject.cpp:23-67)."""
    w1, v1 = (np.ascontiguousarray(bow1[0], np.uint32), np.ascontiguousarray(bow1[1], np.float64))
    w2, v2 = (np.ascontiguousarray(bow2[0], np.uint32), np.ascontiguousarray(bow2[1], np.float64))
    return float(load().orbx_bow_score_l1(ptr(w1), ptr(v1), len(w1), ptr(w2), ptr(v2), len(w2)))


def bow_db_score(query_bow, kf_bows, device: int = 0):
    """Scoring pass of KeyFrameDatabase::DetectRelocalizationCandidates
    (src/KeyFrameDatabase.cc:220-278) on the GPU: for every keyframe BowVector, the number of
    words it shares with the query and (float)L1Scoring::score(query, keyframe)."""
    qw = np.ascontiguousarray(query_bow[0], np.uint32)
    qv = np.ascontiguousarray(query_bow[1], np.float64)
    nkf = len(kf_bows)
    sizes = np.array([len(b[0]) for b in kf_bows], np.int64)
    off = np.zeros(nkf + 1, np.int32)
    np.cumsum(sizes, out=off[1:])
    words = np.concatenate([np.asarray(b[0], np.uint32) for b in kf_bows]) if nkf else np.zeros(0, np.uint32)
    vals = np.concatenate([np.asarray(b[1], np.float64) for b in kf_bows]) if nkf else np.zeros(0)
    common = np.zeros(max(nkf, 1), np.int32)
    score = np.zeros(max(nkf, 1), np.float32)
    check("orbx_bow_db_score", load().orbx_bow_db_score(
        ptr(qw), ptr(qv), len(qw), nkf, ptr(off), ptr(np.ascontiguousarray(words)),
        ptr(np.ascontiguousarray(vals)), ptr(common), ptr(score), device))
    return common[:nkf], score[:nkf]
