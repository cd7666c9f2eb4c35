"""Seeded synthetic grayscale frames (harness data, not part of the hot path).

There are no datasets in the build image (no KITTI/TUM/EuRoC), so tests and bench.py use
frames generated here, as SURVEY.md §8(d) prescribes: piecewise-constant random rectangles
and disks (intensities U[0,255]) over a low-frequency gradient, plus Gaussian noise, clipped
to uint8.  Stereo pairs are rendered from one layered scene: every shape carries a
disparity d in [2, 64] px and the right view draws it shifted left by d (rectified,
row-aligned), nearer shapes painted last; the two views get independent noise.
"""
from __future__ import annotations

import numpy as np

KITTI = dict(width=1241, height=376, nfeatures=2000, fx=718.856, mbf=386.1448)  # KITTI00-02.yaml
TUM = dict(width=640, height=480, nfeatures=1000)                             # TUM1.yaml
EUROC = dict(width=752, height=480, nfeatures=1000)                           # EuRoC.yaml


def _scene(rng, width, height, n_rect, n_disk):
    shapes = []
    for _ in range(n_rect):
        w = int(rng.integers(6, max(7, width // 6)))
        h = int(rng.integers(6, max(7, height // 5)))
        x0 = int(rng.integers(-w // 2, width))
        y0 = int(rng.integers(-h // 2, height))
        shapes.append(("rect", x0, y0, w, h, float(rng.uniform(0, 255)), float(rng.uniform(2, 64))))
    for _ in range(n_disk):
        r = float(rng.uniform(3, max(4, min(width, height) / 10)))
        cx = float(rng.uniform(0, width))
        cy = float(rng.uniform(0, height))
        shapes.append(("disk", cx, cy, r, 0, float(rng.uniform(0, 255)), float(rng.uniform(2, 64))))
    shapes.sort(key=lambda s: s[6])  # far (small disparity) first
    gx, gy, g0 = rng.uniform(-60, 60), rng.uniform(-60, 60), rng.uniform(60, 190)
    return shapes, (gx, gy, g0)


def _render(shapes, grad, width, height, shift_scale):
    gx, gy, g0 = grad
    yy, xx = np.mgrid[0:height, 0:width].astype(np.float32)
    img = g0 + gx * (xx / width - 0.5) + gy * (yy / height - 0.5)
    for kind, a, b, c, d, val, disp in shapes:
        dx = -disp * shift_scale
        if kind == "rect":
            x0 = int(round(a + dx))
            x1, y0, y1 = x0 + c, b, b + d
            x0c, x1c = max(0, x0), min(width, x1)
            y0c, y1c = max(0, y0), min(height, y1)
            if x0c < x1c and y0c < y1c:
                img[y0c:y1c, x0c:x1c] = val
        else:
            cx, cy, r = a + dx, b, c
            xa, xb = max(0, int(cx - r) - 1), min(width, int(cx + r) + 2)
            ya, yb = max(0, int(cy - r) - 1), min(height, int(cy + r) + 2)
            if xa < xb and ya < yb:
                sub = (xx[ya:yb, xa:xb] - cx) ** 2 + (yy[ya:yb, xa:xb] - cy) ** 2 <= r * r
                img[ya:yb, xa:xb][sub] = val
    return img


def frame(seed: int, width: int = 1241, height: int = 376, n_rect: int | None = None,
          n_disk: int | None = None, noise: float = 3.0) -> np.ndarray:
    """One monocular uint8 frame (H x W), deterministic in `seed`."""
    rng = np.random.default_rng(seed)
    area = width * height
    n_rect = n_rect if n_rect is not None else max(8, area // 2500)
    n_disk = n_disk if n_disk is not None else max(4, area // 4000)
    shapes, grad = _scene(rng, width, height, n_rect, n_disk)
    img = _render(shapes, grad, width, height, 0.0)
    img += rng.normal(0.0, noise, size=img.shape).astype(np.float32)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def stereo_pair(seed: int, width: int = 1241, height: int = 376, noise_l: float = 3.0,
                noise_r: float = 2.0):
    """A rectified (left, right) uint8 pair rendered from one layered scene."""
    rng = np.random.default_rng(seed)
    area = width * height
    shapes, grad = _scene(rng, width, height, max(8, area // 2500), max(4, area // 4000))
    left = _render(shapes, grad, width, height, 0.0)
    right = _render(shapes, grad, width, height, 1.0)
    left += rng.normal(0.0, noise_l, size=left.shape).astype(np.float32)
    right += rng.normal(0.0, noise_r, size=right.shape).astype(np.float32)
    to8 = lambda a: np.clip(np.rint(a), 0, 255).astype(np.uint8)
    return to8(left), to8(right)


def edge_cases(width: int = 640, height: int = 480):
    """Named edge-case frames: blank, saturated, checkerboard (score ties), tiny."""
    yy, xx = np.mgrid[0:height, 0:width]
    return {
        "zeros": np.zeros((height, width), np.uint8),
        "white": np.full((height, width), 255, np.uint8),
        "checker8": (((xx // 8 + yy // 8) % 2) * 255).astype(np.uint8),
        "tiny64": frame(7, 64, 64),
    }
