"""my_orb_slam2_amd — MI355X-native ORB front-end (ORB-SLAM2 hot path) on gfx950 HIP kernels.

Host-side mirror of the reference's operator interface for this path:

* ``ORBextractor`` — ORB_SLAM2::ORBextractor (include/ORBextractor.h:45-111)
* ``compute_stereo_matches`` — Frame::ComputeStereoMatches (src/Frame.cc:496-686)
* ``ORBmatcher`` — ORB_SLAM2::ORBmatcher descriptor matching (include/ORBmatcher.h)
* ``Vocabulary`` — ORBVocabulary / DBoW2 transform (Frame::ComputeBoW, src/Frame.cc:420-427)
* ``KeyFrameDatabase`` — ORB_SLAM2::KeyFrameDatabase candidate detection (src/KeyFrameDatabase.cc)

Everything routes through liborbx.so (include/orbx.h).  There is no CPU fallback.
"""
from __future__ import annotations

from ._lib import KEYPOINT_DTYPE, OrbxError, load
from .extractor import ORBextractor, compute_stereo_matches, extract_stereo, StereoBatch
from .matcher import ORBmatcher, descriptor_distance
from .vocabulary import Vocabulary, bow_score_l1
from .kfdb import KeyFrameDatabase

__all__ = ["ORBextractor", "ORBmatcher", "compute_stereo_matches", "extract_stereo", "descriptor_distance",
           "StereoBatch", "Vocabulary", "bow_score_l1", "KeyFrameDatabase", "KEYPOINT_DTYPE", "OrbxError", "load"]
