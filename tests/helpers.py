"""Shared helpers for the parity tests."""
import numpy as np


def assert_kps_equal(got, exp, what=""):
    assert got.shape == exp.shape, f"{what}: {got.shape} keypoints vs oracle {exp.shape}"
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        a, b = got[f], exp[f]
        if a.dtype.kind == "f":
            bad = np.nonzero(a.view(np.uint32) != b.view(np.uint32))[0]
        else:
            bad = np.nonzero(a != b)[0]
        assert bad.size == 0, (f"{what}: field {f} differs at {bad.size} keypoints, first "
                               f"{bad[:5]} got {a[bad[:5]]} exp {b[bad[:5]]}")


def assert_bytes_equal(got, exp, what=""):
    if got is None or exp is None:
        assert got is None and exp is None, f"{what}: one side is None"
        return
    assert got.shape == exp.shape, f"{what}: shape {got.shape} vs {exp.shape}"
    bad = np.nonzero(np.any(got != exp, axis=tuple(range(1, got.ndim))))[0] if got.ndim > 1 \
        else np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{what}: {bad.size} rows differ, first {bad[:5]}"


def assert_f32_bits_equal(got, exp, what=""):
    assert got.shape == exp.shape, f"{what}: shape {got.shape} vs {exp.shape}"
    bad = np.nonzero(got.view(np.uint32) != exp.view(np.uint32))[0]
    assert bad.size == 0, (f"{what}: {bad.size} values differ, first {bad[:5]} "
                           f"got {got[bad[:5]]} exp {exp[bad[:5]]}")
