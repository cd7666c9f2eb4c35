"""GPU parity: ORBextractor / ComputeStereoMatches on the HIP path vs the CPU restatement.

Bit-exact bar: keypoints (every cv::KeyPoint field, bitwise), descriptors, pyramid bytes,
stereo uRight/depth (bitwise float) and the valid-match count.
"""
import numpy as np
import pytest

from helpers import assert_bytes_equal, assert_f32_bits_equal, assert_kps_equal
from my_orb_slam2_amd import synth

pytestmark = pytest.mark.gpu

KITTI_MBF, KITTI_FX = 386.1448, 718.856


def _pair(oracle_mod, nf, sf, nl, ini, mn, simd=1):
    import my_orb_slam2_amd as m
    return (m.ORBextractor(nf, sf, nl, ini, mn, cv_simd=simd),
            oracle_mod.OracleExtractor(nf, sf, nl, ini, mn, simd=simd))


def _check_extract(gpu_ext, ora_ext, img, what):
    k_g, d_g = gpu_ext(img)
    k_o, d_o = ora_ext(img)
    for l in range(ora_ext.nlevels):
        assert_bytes_equal(gpu_ext.pyramid_level(l), ora_ext.level(l), f"{what} pyramid L{l}")
    assert_kps_equal(k_g, k_o, what)
    assert_bytes_equal(d_g, d_o, what + " descriptors")
    return k_g, d_g


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_kitti_extract_parity(oracle_mod, orbx_lib, gpu, seed):
    g, o = _pair(oracle_mod, 2000, 1.2, 8, 20, 7)
    img = synth.frame(seed, 1241, 376)
    k, _ = _check_extract(g, o, img, f"kitti seed {seed}")
    assert 1500 < len(k) <= 2000 + 3 * 8


@pytest.mark.parametrize("size,nf", [((640, 480), 1000), ((752, 480), 1000)])
def test_tum_euroc_extract_parity(oracle_mod, orbx_lib, gpu, size, nf):
    g, o = _pair(oracle_mod, nf, 1.2, 8, 20, 7)
    _check_extract(g, o, synth.frame(11, *size), f"{size}")


@pytest.mark.parametrize("simd", [0, 1])
def test_opencv_rounding_modes(oracle_mod, orbx_lib, gpu, simd):
    g, o = _pair(oracle_mod, 1000, 1.2, 8, 20, 7, simd=simd)
    _check_extract(g, o, synth.frame(5, 640, 480), f"simd={simd}")


@pytest.mark.parametrize("params", [(500, 1.2, 8, 20, 7), (3000, 1.2, 8, 20, 7),
                                    (1000, 1.3, 6, 25, 10), (1500, 1.1, 12, 20, 7),
                                    (1000, 2.0, 3, 20, 7), (1000, 2.5, 3, 20, 7)])
def test_param_sweep(oracle_mod, orbx_lib, gpu, params):
    """One image per call: the pyramid is one k_pyr_chain launch (scale 1.1-1.3), per-level
    launches where the chain does not apply (2.0: the exact 2:1 area path; 2.5: a 4-pixel
    group's taps span more than one v_perm window)."""
    g, o = _pair(oracle_mod, *params)
    _check_extract(g, o, synth.frame(21, 800, 600), f"params {params}")


@pytest.mark.parametrize("name", ["zeros", "white", "checker8", "tiny64"])
def test_edge_images(oracle_mod, orbx_lib, gpu, name):
    g, o = _pair(oracle_mod, 1000, 1.2, 8, 20, 7)
    img = synth.edge_cases()[name]
    _check_extract(g, o, img, name)


@pytest.mark.parametrize("seed", [3, 4])
def test_dense_corners(oracle_mod, orbx_lib, gpu, seed):
    """Uniform noise: thousands of FAST candidates per level, more than k_octree keeps in LDS,
    so every level's DistributeOctTree runs on the global-scratch candidate arrays."""
    g, o = _pair(oracle_mod, 2000, 1.2, 8, 20, 7)
    img = np.random.default_rng(seed).integers(0, 256, (376, 1241), dtype=np.uint8)
    assert len(o(img)[0]) > 0 and len(o.candidates(0)) > 8192
    _check_extract(g, o, img, f"noise seed {seed}")


def test_empty_image(orbx_lib, gpu):
    import my_orb_slam2_amd as m
    g = m.ORBextractor(1000, 1.2, 8, 20, 7)
    assert g(np.zeros((0, 0), np.uint8)) == (None, None)


def _check_stereo(oracle_mod, L, R, params):
    import my_orb_slam2_amd as m
    gl, ol = _pair(oracle_mod, *params)
    gr, orr = _pair(oracle_mod, *params)
    kl, _ = _check_extract(gl, ol, L, "left")
    _check_extract(gr, orr, R, "right")
    mb = np.float32(KITTI_MBF) / np.float32(KITTI_FX)
    u_g, d_g, n_g = m.compute_stereo_matches(gl, gr, KITTI_MBF, float(mb))
    u_o, d_o, n_o = oracle_mod.stereo_match(ol, orr, len(kl), KITTI_MBF, float(mb))
    assert_f32_bits_equal(u_g, u_o, "uRight")
    assert_f32_bits_equal(d_g, d_o, "depth")
    assert n_g == n_o
    return n_g


@pytest.mark.parametrize("seed", [0, 3])
def test_kitti_stereo_parity(oracle_mod, orbx_lib, gpu, seed):
    L, R = synth.stereo_pair(seed)
    assert _check_stereo(oracle_mod, L, R, (2000, 1.2, 8, 20, 7)) > 100


@pytest.mark.parametrize("params,size", [((3000, 1.2, 8, 20, 7), (800, 600)),
                                         ((1500, 1.1, 12, 20, 7), (752, 480)),
                                         ((1000, 2.0, 3, 20, 7), (640, 480)),
                                         ((500, 1.2, 8, 20, 7), (333, 97))])
def test_stereo_param_sweep(oracle_mod, orbx_lib, gpu, params, size):
    """k_stereo's right-keypoint buckets: (octave, row) buckets for the usual sizes; 3000
    features at 800x600 take the row-bucket fallback (the octave buckets and the descriptors
    would exceed the 160 KB of LDS), 12 and 3 levels the octave windows at their edges."""
    L, R = synth.stereo_pair(7, *size)
    assert _check_stereo(oracle_mod, L, R, params) > (50 if size[1] > 200 else 5)


def test_batched_equals_single(oracle_mod, orbx_lib, gpu):
    import torch
    import my_orb_slam2_amd as m
    B = 4
    pairs = [synth.stereo_pair(100 + i) for i in range(B)]
    Ls = torch.from_numpy(np.stack([p[0] for p in pairs])).to(gpu)
    Rs = torch.from_numpy(np.stack([p[1] for p in pairs])).to(gpu)
    sb = m.StereoBatch(B, 2000)
    mb = float(np.float32(KITTI_MBF) / np.float32(KITTI_FX))
    uR, dep, nv = sb(Ls, Rs, KITTI_MBF, mb)
    torch.cuda.synchronize()
    nkp, kps, desc = sb.fetch("left")
    nkpr, kpsr, descr = sb.fetch("right")
    uRh, deph, nvh = uR.cpu().numpy(), dep.cpu().numpy(), nv.cpu().numpy()
    for i in range(B):
        ol = oracle_mod.OracleExtractor(2000, 1.2, 8, 20, 7)
        orr = oracle_mod.OracleExtractor(2000, 1.2, 8, 20, 7)
        k_o, d_o = ol(pairs[i][0])
        kr_o, dr_o = orr(pairs[i][1])
        assert_kps_equal(kpsr[i, :nkpr[i]], kr_o, f"batch item {i} right")
        assert_bytes_equal(descr[i, :nkpr[i]], dr_o, f"batch item {i} right desc")
        n = nkp[i]
        assert_kps_equal(kps[i, :n], k_o, f"batch item {i}")
        assert_bytes_equal(desc[i, :n], d_o, f"batch item {i} desc")
        u_o, d_oo, n_o = oracle_mod.stereo_match(ol, orr, len(k_o), KITTI_MBF, mb)
        assert_f32_bits_equal(uRh[i, :n], u_o, f"batch item {i} uRight")
        assert_f32_bits_equal(deph[i, :n], d_oo, f"batch item {i} depth")
        assert nvh[i] == n_o


def test_strided_unaligned_views(oracle_mod, orbx_lib, gpu):
    """Input rows at an odd stride (1249 B) from a base 3 bytes past an aligned address: every
    row of level 0 starts at a different alignment, which the level-0 strip walk folds into its
    per-row byte selection."""
    import torch
    import my_orb_slam2_amd as m
    B, W, H, pad = 3, 1241, 376, 8
    pairs = [synth.stereo_pair(200 + i) for i in range(B)]
    bigL = torch.zeros((B, H, W + pad), dtype=torch.uint8)
    bigR = torch.zeros((B, H, W + pad), dtype=torch.uint8)
    for i, (l, r) in enumerate(pairs):
        bigL[i, :, 3:3 + W] = torch.from_numpy(l)
        bigR[i, :, 3:3 + W] = torch.from_numpy(r)
    Ls, Rs = bigL.to(gpu)[:, :, 3:3 + W], bigR.to(gpu)[:, :, 3:3 + W]
    assert Ls.stride(1) == W + pad and Ls.storage_offset() == 3
    sb = m.StereoBatch(B, 2000)
    mb = float(np.float32(KITTI_MBF) / np.float32(KITTI_FX))
    sb(Ls, Rs, KITTI_MBF, mb)
    torch.cuda.synchronize()
    nkp, kps, desc = sb.fetch("left")
    nkpr, kpsr, descr = sb.fetch("right")
    for i in range(B):
        for side, (n, k, d) in (("left", (nkp, kps, desc)), ("right", (nkpr, kpsr, descr))):
            o = oracle_mod.OracleExtractor(2000, 1.2, 8, 20, 7)
            k_o, d_o = o(pairs[i][0 if side == "left" else 1])
            assert_kps_equal(k[i, :n[i]], k_o, f"strided item {i} {side}")
            assert_bytes_equal(d[i, :n[i]], d_o, f"strided item {i} {side} desc")


@pytest.mark.parametrize("simd", [0, 1])
def test_blurred_levels_bitwise(oracle_mod, orbx_lib, gpu, simd):
    """Every blurred level vs GaussianBlur(7x7, sigma 2) restated on the same level, including
    saturated images (row sums of 255s drive the column sums past 2^24)."""
    import my_orb_slam2_amd as m
    rng = np.random.default_rng(9)
    sat = np.where(rng.random((376, 1241)) < 0.7, 255, rng.integers(0, 256, (376, 1241))).astype(np.uint8)
    cases = {"kitti": synth.frame(3), "saturated": sat, **synth.edge_cases()}
    g = m.ORBextractor(2000, 1.2, 8, 20, 7, cv_simd=simd)
    for name, img in cases.items():
        g(img)
        for l in range(8):
            lvl = g.pyramid_level(l)
            want = oracle_mod.gaussian7(lvl, simd)
            assert_bytes_equal(g.blur_level(l), want, f"{name} simd={simd} blur L{l}")


def test_batch_blurred_levels_bitwise(oracle_mod, orbx_lib, gpu):
    """The blurred levels of a bench-like batch (96 images: the strip walk's 64 / 32 / 16 /
    8-row strips and its tiled band stores, every wave position of a level) vs
    GaussianBlur(7x7, sigma 2) restated on each image's own level (ORBextractor.cc:1107-1108),
    read back through the de-tiling orbx_blur_level."""
    import torch
    import my_orb_slam2_amd as m
    B = 96
    imgs = np.stack([np.roll(synth.frame(40 + i % 12), 31 * (i // 12), axis=0) for i in range(B)])
    g = m.ORBextractor(2000, 1.2, 8, 20, 7, max_batch=B)
    g.extract_batch_device(torch.from_numpy(imgs).to(gpu))
    torch.cuda.synchronize()
    for i in (0, 1, 37, 95):
        for l in range(8):
            lvl = g.pyramid_level(l, i)
            want = oracle_mod.gaussian7(lvl, True)
            got = g.blur_level(l, i)
            bad = np.argwhere(got != want)
            if bad.size:
                y, x = bad[0]
                y0, x0 = y & ~3, x & ~15
                print("bad", bad.tolist())
                print("got\n", got[y0 - 4:y0 + 8, x0:x0 + 16])
                print("want\n", want[y0 - 4:y0 + 8, x0:x0 + 16])
            assert bad.size == 0, f"image {i} blur L{l} ({lvl.shape}): {len(bad)} pixels differ, first (y, x) {bad[:6].tolist()}"


def test_large_batch_equals_single_images(oracle_mod, orbx_lib, gpu):
    """Batch invariance at a bench-like batch: 48 stereo pairs (96 images: every kernel runs
    its XCD-ordered grid) give, image by image, exactly the single-image outputs; two of them
    are also checked against the CPU restatement (size-independent property, §8 parity).
    The strip heights differ between the two runs (96 images: 64-row strips on levels 0-1,
    32 / 16 / 8 rows below; one image: 8 rows everywhere), so this also pins the strip walk's
    result as independent of its height."""
    import torch
    import my_orb_slam2_amd as m
    B = 48
    base = [synth.stereo_pair(200 + i) for i in range(8)]
    # distinct images: base pair i % 8 rolled down by 29 * (i // 8) rows (still rectified)
    pairs = [tuple(np.roll(base[i % 8][v], 29 * (i // 8), axis=0) for v in (0, 1)) for i in range(B)]
    Ls = torch.from_numpy(np.stack([p[0] for p in pairs])).to(gpu)
    Rs = torch.from_numpy(np.stack([p[1] for p in pairs])).to(gpu)
    sb = m.StereoBatch(B, 2000)
    mb = float(np.float32(KITTI_MBF) / np.float32(KITTI_FX))
    uR, dep, nv = sb(Ls, Rs, KITTI_MBF, mb)
    torch.cuda.synchronize()
    nkp, kps, desc = sb.fetch("left")
    nkpr, kpsr, descr = sb.fetch("right")
    uRh, deph, nvh = uR.cpu().numpy(), dep.cpu().numpy(), nv.cpu().numpy()
    gl, gr = m.ORBextractor(2000, 1.2, 8, 20, 7), m.ORBextractor(2000, 1.2, 8, 20, 7)
    for i in range(B):
        k1, d1 = gl(pairs[i][0])
        k2, d2 = gr(pairs[i][1])
        assert nkp[i] == len(k1) and nkpr[i] == len(k2), f"pair {i} keypoint counts"
        assert_kps_equal(kps[i, :nkp[i]], k1, f"pair {i} left")
        assert_bytes_equal(desc[i, :nkp[i]], d1, f"pair {i} left desc")
        assert_kps_equal(kpsr[i, :nkpr[i]], k2, f"pair {i} right")
        assert_bytes_equal(descr[i, :nkpr[i]], d2, f"pair {i} right desc")
        u1, z1, n1 = m.compute_stereo_matches(gl, gr, KITTI_MBF, mb)
        assert_f32_bits_equal(uRh[i, :nkp[i]], u1, f"pair {i} uRight")
        assert_f32_bits_equal(deph[i, :nkp[i]], z1, f"pair {i} depth")
        assert nvh[i] == n1
    for i in (5, 41):
        ol = oracle_mod.OracleExtractor(2000, 1.2, 8, 20, 7)
        k_o, d_o = ol(pairs[i][0])
        assert_kps_equal(kps[i, :nkp[i]], k_o, f"pair {i} vs oracle")
        assert_bytes_equal(desc[i, :nkp[i]], d_o, f"pair {i} desc vs oracle")


def test_stereo_split_equals_unsplit(orbx_lib, gpu):
    """k_stereo splits a pair's left keypoints over up to four workgroups (median in
    k_stereo_cut) when a call has at most 128 pairs (8 pairs: 4 workgroups each), and keeps one
    workgroup per pair above that: 136 pairs
    in one call (one workgroup per pair) give bit for bit the uRight / depth / counts of the
    same pairs in calls of 8 (split; those are checked against the oracle elsewhere)."""
    import torch
    import my_orb_slam2_amd as m
    B, C = 136, 8
    base = [synth.stereo_pair(400 + i, 640, 200) for i in range(8)]
    pairs = [tuple(np.roll(base[i % 8][v], 13 * (i // 8), axis=0) for v in (0, 1)) for i in range(B)]
    Ls = torch.from_numpy(np.stack([p[0] for p in pairs])).to(gpu)
    Rs = torch.from_numpy(np.stack([p[1] for p in pairs])).to(gpu)
    mb = float(np.float32(KITTI_MBF) / np.float32(KITTI_FX))
    big = m.StereoBatch(B, 1000)
    uR, dep, nv = (t.cpu().numpy() for t in big(Ls, Rs, KITTI_MBF, mb))
    nkp = big.fetch("left")[0]
    # calls of 8 pairs (4 workgroups each) over all 136, and of one pair (the most workgroups
    # per pair: the last one to arrive takes the median, include the hand-off's ordering) over
    # 48 of them
    for C, upto in ((8, B), (1, 48)):
        small = m.StereoBatch(C, 1000)
        for c0 in range(0, upto, C):
            u2, d2, n2 = (t.cpu().numpy() for t in small(Ls[c0:c0 + C], Rs[c0:c0 + C], KITTI_MBF, mb))
            assert np.array_equal(small.fetch("left")[0], nkp[c0:c0 + C]), f"pairs {c0}.. keypoints"
            assert np.array_equal(n2, nv[c0:c0 + C]), f"pairs {c0}.. valid counts"
            for i in range(C):
                n = nkp[c0 + i]
                assert_f32_bits_equal(u2[i, :n], uR[c0 + i, :n], f"pair {c0 + i} uRight")
                assert_f32_bits_equal(d2[i, :n], dep[c0 + i, :n], f"pair {c0 + i} depth")
    assert nv.sum() > 0


def test_stereo_batch_shape_and_size_changes(orbx_lib, gpu):
    """One StereoBatch object across calls of different batch sizes and image shapes: the
    output buffers follow (B, W, H, kp_cap) and fetch() reads the views of the last call
    (right view of pair i = image B + i of that call), each equal to single-image runs."""
    import torch
    import my_orb_slam2_amd as m
    sb = m.StereoBatch(2, 1000)
    gl, gr = m.ORBextractor(1000, 1.2, 8, 20, 7), m.ORBextractor(1000, 1.2, 8, 20, 7)
    mb = float(np.float32(KITTI_MBF) / np.float32(KITTI_FX))
    # small frames first (1 octree root), then wider ones (3 roots: a larger kp_cap), then a
    # smaller batch of the wide shape
    for seed, (w, h), B in ((300, (320, 240), 2), (310, (960, 300), 3), (320, (960, 300), 1)):
        pairs = [synth.stereo_pair(seed + i, w, h) for i in range(B)]
        Ls = torch.from_numpy(np.stack([p[0] for p in pairs])).to(gpu)
        Rs = torch.from_numpy(np.stack([p[1] for p in pairs])).to(gpu)
        uR, dep, nv = sb(Ls, Rs, KITTI_MBF, mb)
        torch.cuda.synchronize()
        kc = sb.ext.batch_view().kp_cap
        assert uR.shape == (B, kc) and dep.shape == (B, kc) and nv.shape == (B,)
        nkp, kps, _ = sb.fetch("left")
        nkpr, kpsr, _ = sb.fetch("right")
        assert len(nkp) == B and len(nkpr) == B
        uRh, nvh = uR.cpu().numpy(), nv.cpu().numpy()
        for i in range(B):
            k1, _ = gl(pairs[i][0])
            k2, _ = gr(pairs[i][1])
            assert_kps_equal(kps[i, :nkp[i]], k1, f"{w}x{h} B={B} pair {i} left")
            assert_kps_equal(kpsr[i, :nkpr[i]], k2, f"{w}x{h} B={B} pair {i} right")
            u1, _, n1 = m.compute_stereo_matches(gl, gr, KITTI_MBF, mb)
            assert_f32_bits_equal(uRh[i, :nkp[i]], u1, f"{w}x{h} B={B} pair {i} uRight")
            assert nvh[i] == n1


@pytest.mark.parametrize("nlevels,resident", [(8, False), (3, False), (8, True)])
def test_overlap_modes_identical(orbx_lib, gpu, nlevels, resident):
    """The side branch (orbx_extractor_set_overlap: the first levels' FAST / octree /
    orientation on a second stream, forked inside the pyramid chain) changes only the
    schedule: every mode, fork level and level count gives the one-stream outputs bit for bit
    (keypoints, descriptors, uRight, depth, counts) on 24 stereo pairs, including fork points
    past the last level and side branches wider than the pyramid."""
    import torch
    import my_orb_slam2_amd as m
    B = 24
    base = [synth.stereo_pair(600 + i) for i in range(6)]
    pairs = [tuple(np.roll(base[i % 6][v], 31 * (i // 6), axis=0) for v in (0, 1)) for i in range(B)]
    Ls = torch.from_numpy(np.stack([p[0] for p in pairs])).to(gpu)
    Rs = torch.from_numpy(np.stack([p[1] for p in pairs])).to(gpu)
    mb = float(np.float32(KITTI_MBF) / np.float32(KITTI_FX))
    sb = m.StereoBatch(B, 2000, 1.2, nlevels, 20, 7)
    if resident:   # images in the level-0 slots: mode 4 moves level 0's launch to the branch
        Lv, Rv = sb.input_views(Ls.shape[2], Ls.shape[1])
        Lv.copy_(Ls)
        Rv.copy_(Rs)

    def run(cfg):
        sb.ext.set_overlap(*cfg)
        res = sb.run_resident(KITTI_MBF, mb) if resident else sb(Ls, Rs, KITTI_MBF, mb)
        outs = [t.cpu().numpy().copy() for t in res]
        torch.cuda.synchronize()
        return outs, sb.fetch("left"), sb.fetch("right")

    ref = run((0, 0, 1))
    assert ref[0][2].sum() > 0
    for cfg in [(-1, 0, 0), (1, 0, 1), (2, 1, 1), (3, 1, 1), (3, 3, 1), (3, 3, 2), (3, 4, 3),
                (3, 9, 1), (3, 2, 12), (4, 0, 1), (4, 1, 1), (4, 3, 1), (4, 2, 2)]:
        got = run(cfg)
        (u0, d0, n0), l0, r0 = ref
        (u1, d1, n1), l1, r1 = got
        assert np.array_equal(n0, n1), f"{cfg}: valid counts"
        for side, a, b in (("left", l0, l1), ("right", r0, r1)):
            assert np.array_equal(a[0], b[0]), f"{cfg}: {side} keypoint counts"
            for i in range(B):
                n = a[0][i]
                assert_kps_equal(b[1][i, :n], a[1][i, :n], f"{cfg} {side} pair {i}")
                assert_bytes_equal(b[2][i, :n], a[2][i, :n], f"{cfg} {side} pair {i} desc")
        for i in range(B):
            n = l0[0][i]
            assert_f32_bits_equal(u1[i, :n], u0[i, :n], f"{cfg} pair {i} uRight")
            assert_f32_bits_equal(d1[i, :n], d0[i, :n], f"{cfg} pair {i} depth")
    sb.ext.set_overlap(-1)


def test_overlap_branch_in_a_hip_graph(orbx_lib, gpu):
    """A stereo call with the side branch (mode 3: the fork / join events between the caller's
    stream and the handle's second stream) captured into a HIP graph and replayed gives the
    eager one-stream outputs bit for bit (the pipelined host-io path replays such graphs)."""
    import torch
    import my_orb_slam2_amd as m
    B, W, H = 8, 1241, 376
    pairs = [synth.stereo_pair(700 + i) for i in range(B)]
    mb = float(np.float32(KITTI_MBF) / np.float32(KITTI_FX))
    sb = m.StereoBatch(B, 2000)
    Lv, Rv = sb.input_views(W, H)
    Lv.copy_(torch.from_numpy(np.stack([p[0] for p in pairs])).to(gpu))
    Rv.copy_(torch.from_numpy(np.stack([p[1] for p in pairs])).to(gpu))
    s = torch.cuda.Stream(gpu)
    sb.ext.set_overlap(0)
    with torch.cuda.stream(s):
        ref = [t.cpu().numpy().copy() for t in sb.run_resident(KITTI_MBF, mb, stream=s.cuda_stream)]
    s.synchronize()
    ref_l, ref_r = sb.fetch("left"), sb.fetch("right")
    sb.ext.set_overlap(3, 3, 1)
    with torch.cuda.stream(s):   # eager run first (workspace and batch view ready)
        sb.run_resident(KITTI_MBF, mb, stream=s.cuda_stream)
    s.synchronize()
    for t in (sb.uR, sb.depth, sb.nvalid):
        t.zero_()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        sb.run_resident(KITTI_MBF, mb, stream=s.cuda_stream)
    for _ in range(2):
        with torch.cuda.stream(s):
            g.replay()
    s.synchronize()
    got = [t.cpu().numpy() for t in (sb.uR, sb.depth, sb.nvalid)]
    got_l, got_r = sb.fetch("left"), sb.fetch("right")
    assert np.array_equal(got[2], ref[2]) and ref[2].sum() > 0
    for a, b_, side in ((ref_l, got_l, "left"), (ref_r, got_r, "right")):
        assert np.array_equal(a[0], b_[0]), side
        for i in range(B):
            n = a[0][i]
            assert_kps_equal(b_[1][i, :n], a[1][i, :n], f"graph {side} {i}")
            assert_bytes_equal(b_[2][i, :n], a[2][i, :n], f"graph {side} {i} desc")
    for i in range(B):
        n = ref_l[0][i]
        assert_f32_bits_equal(got[0][i, :n], ref[0][i, :n], f"graph uRight {i}")
        assert_f32_bits_equal(got[1][i, :n], ref[1][i, :n], f"graph depth {i}")
    sb.ext.set_overlap(-1)


def test_overlap_setting_api(orbx_lib, gpu):
    """orbx_extractor_set_overlap / get_overlap: the built-in default (mode 3, fork before
    level 3, one level), explicit settings read back, mode < 0 restores the default, and
    out-of-range arguments are rejected with ORBX_ERR_INVALID without changing the setting."""
    import my_orb_slam2_amd as m
    from my_orb_slam2_amd._lib import OrbxError
    e = m.ORBextractor(1000, 1.2, 8, 20, 7)
    assert e.overlap() == (3, 3, 1)
    e.set_overlap(0, 0, 1)
    assert e.overlap() == (0, 0, 1)
    e.set_overlap(2, 4, 2)
    assert e.overlap() == (2, 4, 2)
    L = orbx_lib
    for bad in [(5, 3, 1), (3, -1, 1), (3, 3, 0)]:
        assert L.orbx_extractor_set_overlap(e._h, *bad) == -1, bad
        assert e.overlap() == (2, 4, 2)
    assert L.orbx_extractor_set_overlap(None, 0, 0, 1) == -1
    assert L.orbx_extractor_get_overlap(None, None, None, None) == -1
    e.set_overlap(-1)
    assert e.overlap() == (3, 3, 1)
    with pytest.raises(OrbxError):
        e.set_overlap(7)


@pytest.mark.parametrize("params,size", [((2000, 1.2, 8, 20, 7), (1241, 376)),
                                         ((3000, 1.2, 8, 20, 7), (800, 600)),
                                         ((500, 1.2, 8, 20, 7), (333, 97))])
def test_extract_stereo_equals_separate(oracle_mod, orbx_lib, gpu, params, size):
    """The one-call stereo Frame (orbx_stereo_frame_view: both views as a two-image batch on
    ONE handle, the stereo match appended, one graph) equals two extractions on two handles
    + orbx_stereo_match, bit for bit; the handle alternates with single-image extractions and
    a second size (the graphs' keys and the output block's layout follow)."""
    import my_orb_slam2_amd as m
    mb = float(np.float32(KITTI_MBF) / np.float32(KITTI_FX))
    one = m.ORBextractor(*params)
    gl, gr = m.ORBextractor(*params), m.ORBextractor(*params)
    for seed in (40, 41, 42):
        L, R = synth.stereo_pair(seed, *size)
        kl, dl, kr, dr, u, d, nv = m.extract_stereo(one, L, R, KITTI_MBF, mb)
        k1, d1 = gl(L)
        k2, d2 = gr(R)
        u1, dd1, n1 = m.compute_stereo_matches(gl, gr, KITTI_MBF, mb)
        assert_kps_equal(kl, k1, f"seed {seed} left")
        assert_bytes_equal(dl, d1, f"seed {seed} left desc")
        assert_kps_equal(kr, k2, f"seed {seed} right")
        assert_bytes_equal(dr, d2, f"seed {seed} right desc")
        assert_f32_bits_equal(u, u1, f"seed {seed} uRight")
        assert_f32_bits_equal(d, dd1, f"seed {seed} depth")
        assert nv == n1 and (nv > 0 or size[1] < 200)
        # the same handle as a single-image extractor between stereo frames
        k3, d3 = one(L)
        assert_kps_equal(k3, k1, f"seed {seed} single after stereo")
    if size == (1241, 376):
        k_o, d_o = oracle_mod.OracleExtractor(*params)(L)
        assert_kps_equal(kl, k_o, "oracle left")
        assert_bytes_equal(dl, d_o, "oracle left desc")
    # another size on the same handle
    L2, R2 = synth.stereo_pair(43, 640, 480)
    kl, dl, kr, dr, u, d, nv = m.extract_stereo(one, L2, R2, KITTI_MBF, mb)
    k1, d1 = gl(L2)
    gr(R2)
    u1, _, n1 = m.compute_stereo_matches(gl, gr, KITTI_MBF, mb)
    assert_kps_equal(kl, k1, "640x480 left")
    assert_f32_bits_equal(u, u1, "640x480 uRight")
    assert nv == n1


def test_frame_server_mixed_sessions(orbx_lib, gpu):
    """Six sessions (each its own extractor and thread) call orbx_stereo_frame_view at once
    with frames of two sizes and two cameras interleaved: the frame server batches the calls
    that meet (frames of one size and camera per batch, the two block pairs alternating,
    graphs per batch size), and every frame's outputs equal the same frame run alone."""
    import threading
    import my_orb_slam2_amd as m
    params = (2000, 1.2, 8, 20, 7)
    cams = [(KITTI_MBF, float(np.float32(KITTI_MBF) / np.float32(KITTI_FX))),
            (KITTI_MBF * 1.25, float(np.float32(KITTI_MBF * 1.25) / np.float32(KITTI_FX)))]
    jobs = []
    for i in range(6):
        size = (1241, 376) if i % 3 else (640, 480)
        jobs.append((synth.stereo_pair(70 + i, *size), cams[i % 2]))
    solo = m.ORBextractor(*params)
    ref = [m.extract_stereo(solo, L, R, mbf, mb) for (L, R), (mbf, mb) in jobs]
    n_sessions, rounds = 6, 8
    exts = [m.ORBextractor(*params) for _ in range(n_sessions)]
    solo.frame_server_stats(reset=True)
    start = threading.Barrier(n_sessions)
    errors = []

    def session(t):
        try:
            start.wait()
            for k in range(rounds):
                j = (t + k) % len(jobs)
                (L, R), (mbf, mb) = jobs[j]
                got = m.extract_stereo(exts[t], L, R, mbf, mb)
                for a, b, what in zip(got[:6], ref[j][:6], ("kl", "dl", "kr", "dr", "u", "d")):
                    if a.tobytes() != b.tobytes():
                        errors.append(f"session {t} frame {j} {what}")
                if got[6] != ref[j][6]:
                    errors.append(f"session {t} frame {j} n_valid")
        except Exception as e:   # noqa: BLE001 - reported below
            errors.append(f"session {t}: {e!r}")

    threads = [threading.Thread(target=session, args=(t,)) for t in range(n_sessions)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in threads), "a session did not finish"
    assert not errors, errors[:5]
    # the batched path ran: batches of several frames, in both block pairs
    st = solo.frame_server_stats()
    assert st["solo_calls"] + st["served_frames"] == n_sessions * rounds, st
    assert sum(st["batches_of_size"][2:]) > 0, st
    assert min(st["batches_per_pair"]) > 0, st
    assert st["batches"] == sum(st["batches_per_pair"]) == sum(st["batches_of_size"]), st
    assert st["served_frames"] == sum(k * v for k, v in enumerate(st["batches_of_size"])), st
    assert st["users"] >= n_sessions + 1 and st["resident"], st
    assert st["peak_inflight"] >= 1, st


def test_stereo_frame_pyramid_contract(oracle_mod, orbx_lib, gpu):
    """mvImagePyramid after the one-call stereo Frame (include/orbx.h keep_pyramid): six
    sessions at once, so frames are served both alone and in frame-server batches.  With
    keep_pyramid every frame leaves both views' levels on its handle, equal to the reference
    pyramid of ORBextractor.cc:1129-1154 (the oracle's); without it no frame leaves a pyramid
    (ORBX_ERR_STATE), alone or batched.  Then the server's resources are released: explicitly
    while idle, and again when the last session's handle is destroyed."""
    import threading
    import my_orb_slam2_amd as m
    from my_orb_slam2_amd._lib import OrbxError
    params = (1100, 1.2, 8, 20, 7)   # parameters no other test uses: its own frame server
    size = (752, 480)
    mbf = KITTI_MBF
    mb = float(np.float32(mbf) / np.float32(KITTI_FX))
    pairs = [synth.stereo_pair(90 + i, *size) for i in range(3)]
    levels = []
    for L, R in pairs:
        o = [oracle_mod.OracleExtractor(*params), oracle_mod.OracleExtractor(*params)]
        o[0](L)
        o[1](R)
        levels.append([[o[v].level(l) for l in range(8)] for v in range(2)])
    n_sessions, rounds = 6, 6
    exts = [m.ORBextractor(*params) for _ in range(n_sessions)]
    for t, e in enumerate(exts):
        e.keep_pyramid(t % 2 == 0)   # even sessions keep their pyramids, odd ones do not
    exts[0].frame_server_stats(reset=True)
    start = threading.Barrier(n_sessions)
    errors = []

    def session(t):
        try:
            start.wait()
            for k in range(rounds):
                j = (t + k) % len(pairs)
                m.extract_stereo(exts[t], *pairs[j], mbf, mb)
                if t % 2:
                    try:
                        exts[t].pyramid_level(0, 0)
                        errors.append(f"session {t} frame {j}: a pyramid without keep_pyramid")
                    except OrbxError:
                        pass
                    continue
                for v in range(2):
                    for l in range(8):
                        if not np.array_equal(exts[t].pyramid_level(l, v), levels[j][v][l]):
                            errors.append(f"session {t} frame {j} view {v} level {l}")
        except Exception as e:   # noqa: BLE001 - reported below
            errors.append(f"session {t}: {e!r}")

    threads = [threading.Thread(target=session, args=(t,)) for t in range(n_sessions)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in threads), "a session did not finish"
    assert not errors, errors[:5]
    st = exts[0].frame_server_stats()
    assert st["served_frames"] > 0 and st["solo_calls"] + st["served_frames"] == n_sessions * rounds, st
    assert st["resident"] and st["users"] == n_sessions, st
    # explicit release while idle, then a frame recreates the resources
    exts[1].frame_server_release()
    assert not exts[0].frame_server_stats()["resident"]
    m.extract_stereo(exts[2], *pairs[0], mbf, mb)
    assert np.array_equal(exts[2].pyramid_level(3, 1), levels[0][1][3])
    # destroying every session's handle releases the server (the last user goes)
    probe = m.ORBextractor(*params)   # same device and parameters, never a user
    for e in exts:
        e.close()
    st = probe.frame_server_stats()
    assert st["users"] == 0 and not st["resident"], st
