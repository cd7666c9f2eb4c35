"""ORBmatcher over liborbx.so (include/ORBmatcher.h, src/ORBmatcher.cc)."""
from __future__ import annotations

import numpy as np

from ._lib import load, ptr

TH_LOW = 50      # src/ORBmatcher.cc:37
TH_HIGH = 100    # src/ORBmatcher.cc:38
HISTO_LENGTH = 30  # src/ORBmatcher.cc:39


def descriptor_distance(a: np.ndarray, b: np.ndarray) -> int:
    """ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1715-1731)."""
    a = np.ascontiguousarray(a, np.uint8).reshape(32)
    b = np.ascontiguousarray(b, np.uint8).reshape(32)
    return int(load().orbx_descriptor_distance(ptr(a), ptr(b)))


class ORBmatcher:
    """ORB_SLAM2::ORBmatcher(nnratio, checkOri)."""

    TH_LOW = TH_LOW
    TH_HIGH = TH_HIGH
    HISTO_LENGTH = HISTO_LENGTH

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)

    DescriptorDistance = staticmethod(descriptor_distance)
