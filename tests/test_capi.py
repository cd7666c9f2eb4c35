"""CPU: the C-ABI library loads and exports every function include/*.h declares; the
product path refuses to run without a GPU (no silent CPU fallback)."""
import ctypes
import pathlib
import re

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def declared_functions():
    text = "".join(p.read_text() for p in sorted((ROOT / "include").glob("*.h")))
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(orbx_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("orbx_extractor_create", "orbx_extract", "orbx_stereo_match",
                 "orbx_extract_batch_device", "orbx_descriptor_distance",
                 "orbx_matcher_create", "orbx_search_by_bow_kf_frame",
                 "orbx_search_for_triangulation", "orbx_search_by_projection"):
        assert must in names


def test_library_exports_every_declared_symbol(orbx_lib):
    lib = ctypes.CDLL(str(ROOT / "my_orb_slam2_amd" / "liborbx.so"))
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_descriptor_distance_host(orbx_lib):
    import numpy as np
    from my_orb_slam2_amd import descriptor_distance
    rng = np.random.default_rng(0)
    a, b = rng.integers(0, 256, (2, 32), dtype=np.uint8)
    assert descriptor_distance(a, b) == int(np.unpackbits(a ^ b).sum())
    assert descriptor_distance(a, a) == 0


def test_version(orbx_lib):
    assert orbx_lib.orbx_version().startswith(b"orbx")


def test_no_gpu_means_loud_failure(orbx_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    import my_orb_slam2_amd as m
    with pytest.raises(m.OrbxError):
        m.ORBextractor(1000)


def test_three_maxima_host(orbx_lib):
    from my_orb_slam2_amd.matcher import compute_three_maxima
    assert compute_three_maxima([3, 9, 1, 9] + [0] * 26) == (1, 3, 0)
    assert compute_three_maxima([100, 5] + [0] * 28) == (0, -1, -1)


def test_no_gpu_matcher_loud_failure(orbx_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    import my_orb_slam2_amd as m
    with pytest.raises(m.OrbxError):
        m.ORBmatcher(0.75, True)
