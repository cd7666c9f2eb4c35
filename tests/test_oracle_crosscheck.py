"""CPU: check the C++ restatement against independent numpy/pure-Python restatements of the
same published algorithms (small inputs).  Two independent writings of OpenCV's FAST,
resize and GaussianBlur, of DistributeOctTree and of IC_Angle/rBRIEF must agree bit for bit.
"""
import ctypes
import math

import numpy as np
import pytest

from my_orb_slam2_amd import synth

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3),
          (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]   # (dx, dy), cv::FAST order


def _blocky(seed, w, h, noise=4.0):
    rng = np.random.default_rng(seed)
    img = np.full((h, w), 128.0)
    for _ in range(w * h // 60):
        x, y = rng.integers(0, w), rng.integers(0, h)
        img[y:y + rng.integers(2, 8), x:x + rng.integers(2, 8)] = rng.uniform(0, 255)
    img += rng.normal(0, noise, img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def fast_reference(img, t):
    """FAST-9/16 by definition: corner iff 9 contiguous circle pixels are all > v+t or all
    < v-t; score = max over arcs of min |difference| - 1; strict 3x3 NMS on scores."""
    h, w = img.shape
    I = img.astype(int)
    score = np.zeros((h, w), int)
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            v = I[y, x]
            d = [v - I[y + dy, x + dx] for dx, dy in CIRCLE]
            best = -999
            for s in range(16):
                arc = [d[(s + k) % 16] for k in range(9)]
                best = max(best, min(arc), -max(arc))
            if best > t:
                score[y, x] = best - 1
    out = []
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            s = score[y, x]
            if s and all(s > score[y + j, x + i] for j in (-1, 0, 1) for i in (-1, 0, 1)
                         if (i or j)):
                out.append((x, y, s))
    return out


@pytest.mark.parametrize("seed,t", [(0, 7), (1, 20), (2, 12), (3, 0)])
def test_fast_matches_definition(oracle_mod, seed, t):
    img = _blocky(seed, 48, 40)
    got = oracle_mod.fast(img, t)
    exp = fast_reference(img, t)
    assert [(int(k["x"]), int(k["y"]), int(k["response"])) for k in got] == exp
    assert len(exp) > 5 or t == 0


def resize_reference(src, dw, dh, simd):
    sh, sw = src.shape
    if (sw, sh) == (dw, dh):
        return src.copy()
    sx_ = 1.0 / (dw / sw)
    sy_ = 1.0 / (dh / sh)
    if abs(sx_ - round(sx_)) < 2.2e-16 and abs(sy_ - round(sy_)) < 2.2e-16 and \
            round(sx_) == 2 and round(sy_) == 2:
        s = src.astype(int)
        return ((s[0::2, 0::2][:dh, :dw] + s[0::2, 1::2][:dh, :dw] + s[1::2, 0::2][:dh, :dw] +
                 s[1::2, 1::2][:dh, :dw] + 2) >> 2).astype(np.uint8)

    def coefs(n_dst, n_src, scale, clamp):
        ofs, a = [], []
        xmax = n_dst
        for d in range(n_dst):
            f = np.float32((d + 0.5) * scale - 0.5)
            s = int(math.floor(f))
            f = np.float32(f - np.float32(s))
            if clamp:
                if s < 0:
                    f, s = np.float32(0), 0
                if s + 1 >= n_src:
                    xmax = min(xmax, d)
                    if s >= n_src - 1:
                        f, s = np.float32(0), n_src - 1
            ofs.append(s)
            a.append((int(np.rint(np.float32(np.float32(1) - f) * np.float32(2048))),
                      int(np.rint(f * np.float32(2048)))))
        return ofs, a, xmax

    xo, xa, xmax = coefs(dw, sw, sx_, True)
    yo, yb, _ = coefs(dh, sh, sy_, False)
    S = src.astype(np.int64)
    out = np.zeros((dh, dw), np.uint8)
    if simd:
        xs = 0
        while xs <= dw - 16:
            xs += 16
        while xs < dw - 4:
            xs += 4
    else:
        xs = 0
    for y in range(dh):
        r0 = min(max(yo[y], 0), sh - 1)
        r1 = min(max(yo[y] + 1, 0), sh - 1)
        b0, b1 = yb[y]
        for x in range(dw):
            s = xo[x]
            if x < xmax:
                h0 = S[r0, s] * xa[x][0] + S[r0, s + 1] * xa[x][1]
                h1 = S[r1, s] * xa[x][0] + S[r1, s + 1] * xa[x][1]
            else:
                h0, h1 = S[r0, s] * 2048, S[r1, s] * 2048
            if x < xs:
                v = (((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16)
                v = (v + 2) >> 2
            else:
                v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22
            out[y, x] = min(max(v, 0), 255)
    return out


@pytest.mark.parametrize("simd", [0, 1])
@pytest.mark.parametrize("shape", [((60, 50), (50, 42)), ((37, 29), (31, 24)),
                                   ((40, 30), (20, 15)), ((33, 21), (40, 25))])
def test_resize_matches_restatement(oracle_mod, simd, shape):
    (sw, sh), (dw, dh) = shape
    src = synth.frame(9, sw, sh)
    assert np.array_equal(oracle_mod.resize(src, dw, dh, simd), resize_reference(src, dw, dh, simd))


def gaussian_reference(src, simd):
    taps = np.array([18, 34, 49, 55, 49, 34, 18], np.int64)
    p = np.pad(src.astype(np.int64), 3, mode="reflect")      # numpy reflect == REFLECT_101
    h, w = src.shape
    R = sum(taps[k] * p[:, k:k + w] for k in range(7))         # (h+6, w)
    c0 = R[3:3 + h]
    pairs = [R[3 + k:3 + k + h] + R[3 - k:3 - k + h] for k in (1, 2, 3)]
    f = [np.float32(t) * np.float32(1.0 / 65536.0) for t in (55, 49, 34, 18)]
    s = c0.astype(np.float32) * f[0] + np.float32(0)
    for k in range(3):
        s = s + pairs[k].astype(np.float32) * f[k + 1]
    vf = np.clip(np.rint(s), 0, 255).astype(np.uint8)
    vi = np.clip((55 * c0 + sum(taps[4 + k] * pairs[k] for k in range(3)) + 32768) >> 16, 0, 255)
    out = vi.astype(np.uint8)
    if simd:
        xs = (w // 4) * 4
        out[:, :xs] = vf[:, :xs]
    return out


@pytest.mark.parametrize("simd", [0, 1])
@pytest.mark.parametrize("size", [(64, 48), (37, 23), (9, 7)])
def test_gaussian_matches_restatement(oracle_mod, simd, size):
    src = synth.frame(3, *size)
    assert np.array_equal(oracle_mod.gaussian7(src, simd), gaussian_reference(src, simd))


def octree_reference(cands, minX, maxX, minY, maxY, N):
    """DistributeOctTree (src/ORBextractor.cc:539-765) on Python lists; node identity
    = allocation sequence number (the documented tie-break)."""
    if not cands:
        return []
    seq = [0]
    nIni = int(np.round(np.float32(maxX - minX) / np.float32(maxY - minY)))
    if nIni < 1:
        return []
    hX = np.float32(maxX - minX) / np.float32(nIni)

    def node(x0, y0, x1, y1, keys):
        seq[0] += 1
        return {"r": (x0, y0, x1, y1), "k": keys, "more": len(keys) != 1, "seq": seq[0]}

    roots = [node(int(hX * np.float32(i)), 0, int(hX * np.float32(i + 1)), maxY - minY, [])
             for i in range(nIni)]
    for c in cands:
        roots[int(np.float32(c[0]) / hX)]["k"].append(c)
    for r in roots:
        r["more"] = len(r["k"]) != 1
    lst = [r for r in roots if r["k"]]

    def divide(n):
        x0, y0, x1, y1 = n["r"]
        hx = int(math.ceil(np.float32(x1 - x0) / np.float32(2)))
        hy = int(math.ceil(np.float32(y1 - y0) / np.float32(2)))
        sx, sy = x0 + hx, y0 + hy
        rects = [(x0, y0, sx, sy), (sx, y0, x1, sy), (x0, sy, sx, y1), (sx, sy, x1, y1)]
        parts = [[], [], [], []]
        for c in n["k"]:
            parts[(0 if c[1] < sy else 2) if c[0] < sx else (1 if c[1] < sy else 3)].append(c)
        return [(rects[q], parts[q]) for q in range(4)]

    finish = False
    while not finish:
        prev = len(lst)
        new_front, rest, vsize = [], [], []
        for n in lst:
            if not n["more"]:
                rest.append(n)
                continue
            for rect, keys in divide(n):
                if keys:
                    ch = node(*rect, keys)
                    new_front.insert(0, ch)
                    if len(keys) > 1:
                        vsize.append(ch)
        lst = new_front + rest
        if len(lst) >= N or len(lst) == prev:
            finish = True
        elif len(lst) + 3 * len(vsize) > N:
            while not finish:
                prev = len(lst)
                order = sorted(vsize, key=lambda n: (len(n["k"]), n["seq"]))
                vsize = []
                for n in reversed(order):
                    kids = []
                    for rect, keys in divide(n):
                        if keys:
                            ch = node(*rect, keys)
                            kids.insert(0, ch)
                            if len(keys) > 1:
                                vsize.append(ch)
                    lst = kids + [m for m in lst if m is not n]
                    if len(lst) >= N:
                        break
                if len(lst) >= N or len(lst) == prev:
                    finish = True
    out = []
    for n in lst:
        best = n["k"][0]
        for c in n["k"][1:]:
            if c[2] > best[2]:
                best = c
        out.append(best)
    return out


@pytest.mark.parametrize("seed,size,nf", [(0, (1241, 376), 2000), (4, (640, 480), 1000),
                                          (8, (500, 300), 300)])
def test_octree_matches_list_restatement(oracle_mod, seed, size, nf):
    e = oracle_mod.OracleExtractor(nf, 1.2, 8, 20, 7)
    e(synth.frame(seed, *size))
    quotas = e.tables()["features_per_level"]
    for l in range(8):
        w, h = e.level_size(l)
        c = e.candidates(l)
        cands = [(int(k["x"]), int(k["y"]), float(k["response"])) for k in c]
        exp = octree_reference(cands, 16, w - 16, 16, h - 16, int(quotas[l]))
        got = e.level_keypoints(l)
        assert [(int(k["x"]) - 16, int(k["y"]) - 16, float(k["response"])) for k in got] == \
            [(x, y, r) for x, y, r in exp], f"level {l}"


def test_orientation_and_descriptor_restatement(oracle_mod):
    libm = ctypes.CDLL("libm.so.6")
    libm.cosf.restype = libm.sinf.restype = ctypes.c_float
    libm.cosf.argtypes = libm.sinf.argtypes = [ctypes.c_float]
    pat = []
    import pathlib
    for line in (pathlib.Path(__file__).resolve().parents[1] /
                 "my_orb_slam2_amd/csrc/orbx_pattern.inc").read_text().splitlines():
        if not line.startswith("//"):
            pat += [int(v) for v in line.replace(",", " ").split()]
    pat = np.array(pat).reshape(512, 2)
    umax = [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    e = oracle_mod.OracleExtractor(500, 1.2, 8, 20, 7)
    kps, desc = e(synth.frame(2, 640, 480))
    f32 = np.float32
    n_checked = 0
    offset = 0
    for l in range(8):
        lk = e.level_keypoints(l)
        img = e.level(l).astype(int)
        blur = e.level(l, blurred=True)
        for i, k in enumerate(lk[::7]):
            x, y = int(k["x"]), int(k["y"])
            m10 = sum(u * img[y, x + u] for u in range(-15, 16))
            m01 = 0
            for v in range(1, 16):
                vs = 0
                for u in range(-umax[v], umax[v] + 1):
                    p, m = img[y + v, x + u], img[y - v, x + u]
                    vs += p - m
                    m10 += u * (p + m)
                m01 += v * vs
            ang = oracle_mod.fast_atan2(float(m01), float(m10))
            assert f32(ang) == k["angle"]
            a_ = f32(ang) * f32(math.pi / 180.0)
            ca, sa = f32(libm.cosf(a_)), f32(libm.sinf(a_))
            bits = []
            for j in range(256):
                vals = []
                for q in (2 * j, 2 * j + 1):
                    px, py = f32(pat[q, 0]), f32(pat[q, 1])
                    ry = int(np.rint(f32(px * sa) + f32(py * ca)))
                    rx = int(np.rint(f32(px * ca) - f32(py * sa)))
                    vals.append(int(blur[y + ry, x + rx]))
                bits.append(1 if vals[0] < vals[1] else 0)
            d = np.packbits(np.array(bits, np.uint8), bitorder="little")
            assert np.array_equal(d, desc[offset + 7 * i]), f"level {l} kp {7 * i}"
            n_checked += 1
        offset += len(lk)
    assert n_checked > 50
