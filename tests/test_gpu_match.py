"""GPU parity of the descriptor matchers (src/ORBmatcher.cc) against the CPU restatement.

Bit-exact bar: every returned feature index and every match count equal the oracle's on the
same seeded feature sets (synthetic correlated frames with duplicated descriptors for
distance ties, claimed masks, rotation outliers; see my_orb_slam2_amd/synth.py).
"""
import numpy as np
import pytest

from my_orb_slam2_amd import synth
from my_orb_slam2_amd.features import (PROJ_FRAME_MAPPOINTS, PROJ_FUSE, PROJ_FUSE_SCW,
                                       PROJ_KEYFRAME, PROJ_KF_SCW, PROJ_LAST_FRAME, PROJ_SIM3,
                                       FeatureSet, feature_vector)

pytestmark = pytest.mark.gpu


def _matcher(ratio, ori):
    from my_orb_slam2_amd import ORBmatcher
    return ORBmatcher(ratio, ori)


@pytest.mark.parametrize("seed,ratio,ori,single,n", [
    (0, 0.75, True, False, 1000), (1, 0.6, False, False, 2000), (2, 0.7, True, True, 900),
    (3, 0.75, True, True, 1500),   # single node above 1024 candidates: re-read path
    (4, 0.9, True, False, 300)])
def test_bow_kf_frame(oracle_mod, orbx_lib, gpu, seed, ratio, ori, single, n):
    from oracle import matcher as om
    f1, f2, _ = synth.feature_pair(seed, n1=n, n2=n, single_node=single)
    valid = np.random.default_rng(seed).random(f1.n) < 0.85
    m = _matcher(ratio, ori)
    n_g, m_g = m.SearchByBoW(f1, valid, f2)
    n_o, m_o = om.search_by_bow_kf_frame(f1, valid, f2, ratio, ori)
    assert n_g == n_o and n_o > 0
    np.testing.assert_array_equal(m_g, m_o)


@pytest.mark.parametrize("seed,ratio,ori,single", [(0, 0.75, True, False),
                                                   (1, 0.75, False, True)])
def test_bow_kf_kf(oracle_mod, orbx_lib, gpu, seed, ratio, ori, single):
    from oracle import matcher as om
    f1, f2, _ = synth.feature_pair(seed + 20, n1=1200, n2=1000, single_node=single)
    rng = np.random.default_rng(seed)
    v1, v2 = rng.random(f1.n) < 0.8, rng.random(f2.n) < 0.8
    m = _matcher(ratio, ori)
    n_g, m_g = m.SearchByBoW(f1, v1, f2, v2, f_is_keyframe=True)
    n_o, m_o = om.search_by_bow_kf_kf(f1, v1, f2, v2, ratio, ori)
    assert n_g == n_o and n_o > 0
    np.testing.assert_array_equal(m_g, m_o)


@pytest.mark.parametrize("seed,only_stereo,ori,single", [(0, False, False, False),
                                                         (1, True, False, False),
                                                         (2, False, True, False),
                                                         (3, False, False, True)])
def test_triangulation(oracle_mod, orbx_lib, gpu, seed, only_stereo, ori, single):
    from oracle import matcher as om
    k1, k2, F, epi, _ = synth.keyframe_pair(seed, n1=2000, n2=2000, single_node=single)
    rng = np.random.default_rng(seed + 1)
    h1, h2 = rng.random(k1.n) < 0.3, rng.random(k2.n) < 0.3
    s, s2, _ = synth.scale_tables()
    m = _matcher(0.6, ori)
    n_g, p_g = m.SearchForTriangulation(k1, h1, k2, h2, F, epi, s2, s, only_stereo)
    n_o, p_o = om.search_for_triangulation(k1, h1, k2, h2, F, epi, s2, s, only_stereo, ori)
    assert n_g == n_o and n_o > 0
    np.testing.assert_array_equal(p_g, p_o)


PROJ_CASES = [(PROJ_FRAME_MAPPOINTS, 0, 3.0), (PROJ_FRAME_MAPPOINTS, 1, 15.0),
              (PROJ_KF_SCW, 2, 10.0), (PROJ_LAST_FRAME, 3, 7.0), (PROJ_LAST_FRAME, 4, 25.0),
              (PROJ_KEYFRAME, 5, 10.0), (PROJ_FUSE, 6, 3.0), (PROJ_FUSE_SCW, 7, 5.0),
              (PROJ_SIM3, 8, 7.5)]


@pytest.mark.parametrize("mode,seed,th", PROJ_CASES)
def test_projection(oracle_mod, orbx_lib, gpu, mode, seed, th):
    """Large radii (th 15-25) make MapPoints compete for the same features, so the greedy
    claims fall back to the re-scan path often."""
    from oracle import matcher as om
    f1, f2, t = synth.feature_pair(seed + 40, n1=1500, n2=1200, dup_frac=0.1)
    q, d = synth.projection_queries(seed, f1, f2, t, th=th,
                                    mode_levels="frame" if mode in (0, 2, 3) else "kf")
    claimed = np.random.default_rng(seed).random(f2.n) < 0.1
    _, _, isg = synth.scale_tables()
    m = _matcher(0.8, True)
    n_g, m_g = m.search_by_projection(mode, f2, q, d, claimed, isg, orb_dist=64)
    n_o, m_o = om.search_by_projection(mode, f2, q, d, claimed, isg, orb_dist=64, nnratio=0.8)
    assert n_g == n_o and n_o > 0
    np.testing.assert_array_equal(m_g, m_o)


@pytest.mark.parametrize("mode", [PROJ_FRAME_MAPPOINTS, PROJ_KEYFRAME])
def test_projection_large_target(oracle_mod, orbx_lib, gpu, mode):
    """A target of 32000 features: the claim replay runs without the per-feature owner
    words (one query per round), and dense windows overflow the 8-candidate lists."""
    from oracle import matcher as om
    f1, f2, t = synth.feature_pair(77, n1=3000, n2=32000, dup_frac=0.1)
    q, d = synth.projection_queries(5, f1, f2, t, th=6.0)
    claimed = np.random.default_rng(5).random(f2.n) < 0.1
    m = _matcher(0.8, True)
    n_g, m_g = m.search_by_projection(mode, f2, q, d, claimed, orb_dist=64)
    n_o, m_o = om.search_by_projection(mode, f2, q, d, claimed, None, orb_dist=64, nnratio=0.8)
    assert n_g == n_o and n_o > 0
    np.testing.assert_array_equal(m_g, m_o)


@pytest.mark.parametrize("mode,seed,th,prefilter", [
    (PROJ_FRAME_MAPPOINTS, 11, 15.0, False), (PROJ_LAST_FRAME, 12, 7.0, True),
    (PROJ_LAST_FRAME, 13, 25.0, True), (PROJ_KEYFRAME, 15, 10.0, True)])
def test_projection_no_claim_queries(oracle_mod, orbx_lib, gpu, mode, seed, th, prefilter):
    """orbx_search_by_projection_ex: a third of the queries are MapPoints without
    observations (ORBX_QF_NO_CLAIM), whose matches later queries may take over (ORBmatcher.cc
    :90-92, :1471-1473), with and without the rotation filter."""
    from oracle import matcher as om
    f1, f2, t = synth.feature_pair(seed + 40, n1=1500, n2=1200, dup_frac=0.1)
    q, d = synth.projection_queries(seed, f1, f2, t, th=th,
                                    mode_levels="frame" if mode in (0, 2, 3) else "kf")
    rng = np.random.default_rng(seed)
    claimed = rng.random(f2.n) < 0.1
    qflags = (rng.random(len(q)) < 0.33).astype(np.uint8)
    # the first 300 queries once more in front, as MapPoints without observations: their
    # matches stay unclaimed, so the same queries later take those features again
    q, d = np.concatenate([q[:300], q]), np.concatenate([d[:300], d])
    qflags = np.concatenate([np.ones(300, np.uint8), qflags])
    m = _matcher(0.8, True)
    n_g, m_g = m.search_by_projection_ex(mode, f2, q, d, qflags, claimed, orb_dist=64,
                                         prefilter=prefilter)
    n_o, m_o = om.search_by_projection_ex(mode, f2, q, d, qflags, claimed, orb_dist=64,
                                          nnratio=0.8, prefilter=prefilter)
    assert n_g == n_o and n_o > 0
    np.testing.assert_array_equal(m_g, m_o)
    if mode != PROJ_KEYFRAME:   # some feature is matched by two queries
        hit = m_o[m_o >= 0]
        assert len(np.unique(hit)) < len(hit) - 50


def test_projection_no_claim_last_frame_needs_prefilter(oracle_mod, orbx_lib, gpu):
    """LAST_FRAME + rotation check + no-claim queries without ORBX_PROJ_PREFILTER is refused
    by the library and the oracle alike: the reference's rotation filter clears per feature
    (ORBmatcher.cc:1516-1535) and a feature matched by two queries sits in two bins."""
    from my_orb_slam2_amd import OrbxError
    from oracle import matcher as om
    f1, f2, t = synth.feature_pair(54, n1=600, n2=500, dup_frac=0.1)
    q, d = synth.projection_queries(14, f1, f2, t, th=25.0, mode_levels="frame")
    qflags = np.zeros(len(q), np.uint8)
    qflags[3] = 1
    m = _matcher(0.8, True)
    with pytest.raises(OrbxError):
        m.search_by_projection_ex(PROJ_LAST_FRAME, f2, q, d, qflags, orb_dist=64)
    n_o, _ = om.search_by_projection_ex(PROJ_LAST_FRAME, f2, q, d, qflags, orb_dist=64, nnratio=0.8)
    assert n_o == -1
    # without no-claim queries, or with the prefilter, the call runs
    n_g, m_g = m.search_by_projection_ex(PROJ_LAST_FRAME, f2, q, d, np.zeros(len(q), np.uint8),
                                         orb_dist=64)
    n_o, m_o = om.search_by_projection_ex(PROJ_LAST_FRAME, f2, q, d, np.zeros(len(q), np.uint8),
                                          orb_dist=64, nnratio=0.8)
    assert n_g == n_o and n_o > 0
    np.testing.assert_array_equal(m_g, m_o)


def test_sim3(oracle_mod, orbx_lib, gpu):
    from oracle import matcher as om
    f1, f2, t = synth.feature_pair(60, n1=1000, n2=1000)
    q12, d1 = synth.projection_queries(1, f1, f2, t, th=7.5, mode_levels="kf")
    inv = np.full(f2.n, -1, np.int64)
    inv[t[t >= 0]] = np.nonzero(t >= 0)[0]
    q21, d2 = synth.projection_queries(2, f2, f1, inv, th=7.5, mode_levels="kf")
    m = _matcher(0.75, True)
    n_g, m_g = m.SearchBySim3(f1, f2, d1, q12, d2, q21)
    n_o, m_o = om.search_by_sim3(f1, f2, d1, q12, d2, q21)
    assert n_g == n_o and n_o > 0
    np.testing.assert_array_equal(m_g, m_o)


@pytest.mark.parametrize("seed,window,ori", [(0, 100, True), (1, 50, False)])
def test_initialization(oracle_mod, orbx_lib, gpu, seed, window, ori):
    from oracle import matcher as om
    f1, f2, t = synth.feature_pair(70 + seed, n1=2000, n2=2000, dup_frac=0.1)
    prev = np.ascontiguousarray(np.stack([f1.keys["x"], f1.keys["y"]], 1), np.float32)
    p_g, p_o = prev.copy(), prev.copy()
    m = _matcher(0.9, ori)
    n_g, m_g = m.SearchForInitialization(f1, f2, p_g, window)
    n_o, m_o = om.search_for_initialization(f1, f2, p_o, window, 0.9, ori)
    assert n_g == n_o and n_o > 0
    np.testing.assert_array_equal(m_g, m_o)
    np.testing.assert_array_equal(p_g.view(np.int32), p_o.view(np.int32))


def test_empty_and_disjoint(oracle_mod, orbx_lib, gpu):
    from oracle import matcher as om
    f1, f2, _ = synth.feature_pair(80, n1=200, n2=200)
    empty = FeatureSet(f2.keys[:0], f2.desc[:0], f2.u_right[:0], feature_vector(np.zeros(0)),
                       f2.grid)
    empty.grid = synth.feature_pair(80, n1=0, n2=1)[0].grid
    m = _matcher(0.75, True)
    n, mm = m.SearchByBoW(f1, np.ones(f1.n), empty)
    assert n == 0 and len(mm) == 0
    n, mm = m.SearchByBoW(empty, np.ones(0), f1)
    assert n == 0 and (mm == -1).all()
    # no shared FeatureVector node
    g = FeatureSet(f2.keys, f2.desc, f2.u_right, feature_vector(np.full(f2.n, 5)), f2.grid)
    n, mm = m.SearchByBoW(f1, np.ones(f1.n), g)
    assert n == om.search_by_bow_kf_frame(f1, np.ones(f1.n), g, 0.75, True)[0] == 0
    q, d = synth.projection_queries(0, f1, f2, np.full(f1.n, -1), th=3.0)
    n, mm = m.search_by_projection(PROJ_FRAME_MAPPOINTS, empty, q, d)
    assert n == 0 and (mm == -1).all()


def test_batch_relocalisation(oracle_mod, orbx_lib, gpu):
    """SearchByBoW(KeyFrame*, Frame&) of 24 keyframes against one frame, device batch."""
    import torch
    from oracle import matcher as om
    from my_orb_slam2_amd.matcher import DeviceFeatureSet, DeviceKfDb
    frame = synth.feature_pair(90, n1=1000, n2=10)[0]
    kfs, valids = [], []
    for k in range(24):
        kf = synth.feature_pair(100 + k, n1=800 + 20 * k, n2=1000, single_node=(k % 3 == 0))[1]
        # make some keyframes share features with the frame
        src = np.random.default_rng(k).choice(frame.n, 300, replace=False)
        kf.desc[:300] = frame.desc[src]
        from my_orb_slam2_amd.synth import _node_of
        nodes = np.zeros(kf.n, np.int64) if k % 3 == 0 else _node_of(kf.desc, 40)
        kf.fvec = feature_vector(nodes)
        kfs.append(kf)
        valids.append(np.random.default_rng(k + 5).random(kf.n) < 0.9)
    fr = frame
    if True:
        fr.fvec = feature_vector(_node_of(fr.desc, 40))
    m = _matcher(0.75, True)
    db = DeviceKfDb(kfs, valids, gpu)
    df = DeviceFeatureSet(fr, gpu)
    out = torch.full((len(kfs), fr.n), -7, dtype=torch.int32, device=gpu)
    cnt = torch.zeros(len(kfs), dtype=torch.int32, device=gpu)
    m.search_by_bow_kf_frame_batch_device(db.c, df.c, out, cnt)
    m.sync()
    out, cnt = out.cpu().numpy(), cnt.cpu().numpy()
    for k, kf in enumerate(kfs):
        # the single-node keyframes only meet the frame's features at a shared node id
        n_o, m_o = om.search_by_bow_kf_frame(kf, valids[k], fr, 0.75, True)
        assert cnt[k] == n_o, k
        np.testing.assert_array_equal(out[k], m_o)
    assert cnt.sum() > 0


def test_batch_triangulation(oracle_mod, orbx_lib, gpu):
    import torch
    from oracle import matcher as om
    from my_orb_slam2_amd.matcher import DeviceKfDb
    s, s2, _ = synth.scale_tables()
    kfs, flags, jobs, Fs, epis, refs = [], [], [], [], [], []
    for j in range(12):
        k1, k2, F, epi, _ = synth.keyframe_pair(200 + j, n1=1500, n2=1400,
                                                single_node=(j % 4 == 0))
        rng = np.random.default_rng(j)
        h1, h2 = rng.random(k1.n) < 0.3, rng.random(k2.n) < 0.3
        kfs += [k1, k2]
        flags += [h1, h2]
        jobs.append((2 * j, 2 * j + 1))
        Fs.append(F.reshape(9))
        epis.append(epi)
        refs.append(om.search_for_triangulation(k1, h1, k2, h2, F, epi, s2, s, False, False))
    m = _matcher(0.6, False)
    db = DeviceKfDb(kfs, flags, gpu)
    jobs = np.array(jobs, np.int32)
    n1 = np.array([kfs[a].n for a, _ in jobs], np.int32)
    job_off = np.concatenate([[0], np.cumsum(n1)]).astype(np.int32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    out = torch.full((int(job_off[-1]),), -7, dtype=torch.int32, device=gpu)
    cnt = torch.zeros(len(jobs), dtype=torch.int32, device=gpu)
    m.search_for_triangulation_batch_device(db.c, T(jobs[:, 0]), T(jobs[:, 1]),
                                            T(np.array(Fs, np.float32)),
                                            T(np.array(epis, np.float32)), s2, s, T(job_off),
                                            out, cnt)
    m.sync()
    out, cnt = out.cpu().numpy(), cnt.cpu().numpy()
    for j, (n_o, p_o) in enumerate(refs):
        seg = out[job_off[j]:job_off[j + 1]]
        idx1 = np.nonzero(seg >= 0)[0]
        assert cnt[j] == n_o
        np.testing.assert_array_equal(np.stack([idx1, seg[idx1]], 1), p_o)


@pytest.mark.parametrize("mode", [PROJ_FRAME_MAPPOINTS, PROJ_LAST_FRAME, PROJ_KEYFRAME,
                                  PROJ_FUSE, PROJ_KF_SCW])
def test_batch_projection(oracle_mod, orbx_lib, gpu, mode):
    """One projection search per frame over 10 frames of different sizes (one of them empty
    of queries), against the oracle frame by frame."""
    import torch
    from oracle import matcher as om
    from my_orb_slam2_amd.matcher import DeviceFrameBatch
    _, _, isg = synth.scale_tables()
    frames, qs, ds, cls, refs = [], [], [], [], []
    for j in range(10):
        f1, f2, t = synth.feature_pair(300 + j, n1=600 + 97 * j, n2=500 + 131 * j,
                                       dup_frac=0.1)
        q, d = synth.projection_queries(j, f1, f2, t, th=12.0,
                                        mode_levels="frame" if mode in (0, 2, 3) else "kf")
        if j == 4:
            q, d = q[:0], d[:0]
        cl = np.random.default_rng(j).random(f2.n) < 0.1
        frames.append(f2)
        qs.append(q)
        ds.append(d)
        cls.append(cl)
        refs.append(om.search_by_projection(mode, f2, q, d, cl, isg, orb_dist=64, nnratio=0.8))
    m = _matcher(0.8, True)
    fb = DeviceFrameBatch(frames, gpu)
    q_off = np.concatenate([[0], np.cumsum([len(q) for q in qs])]).astype(np.int32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(gpu)
    d_q, d_d = T(np.concatenate(qs)), T(np.concatenate(ds))
    out = torch.full((int(q_off[-1]),), -7, dtype=torch.int32, device=gpu)
    cnt = torch.full((len(frames),), -7, dtype=torch.int32, device=gpu)
    m.search_by_projection_batch_device(mode, fb, d_d, d_q, torch.from_numpy(q_off).to(gpu),
                                        out, cnt, T(np.concatenate(cls).astype(np.uint8)),
                                        isg, orb_dist=64)
    m.sync()
    out, cnt = out.cpu().numpy(), cnt.cpu().numpy()
    for j, (n_o, m_o) in enumerate(refs):
        assert cnt[j] == n_o, j
        np.testing.assert_array_equal(out[q_off[j]:q_off[j + 1]], m_o)
    assert cnt.sum() > 0


def test_batch_projection_capacity(oracle_mod, orbx_lib, gpu):
    """A frame above the declared max_feat is flagged (ORBX_ERR_CAPACITY at sync) and gets no
    matches; the others are unaffected."""
    import torch
    from oracle import matcher as om
    from my_orb_slam2_amd._lib import OrbxError
    from my_orb_slam2_amd.matcher import DeviceFrameBatch
    frames, qs, ds = [], [], []
    for j in range(3):
        f1, f2, t = synth.feature_pair(400 + j, n1=500, n2=400 + 300 * j)
        q, d = synth.projection_queries(j, f1, f2, t, th=5.0)
        frames.append(f2)
        qs.append(q)
        ds.append(d)
    m = _matcher(0.8, True)
    fb = DeviceFrameBatch(frames, gpu)
    fb.max_feat = frames[1].n
    q_off = np.concatenate([[0], np.cumsum([len(q) for q in qs])]).astype(np.int32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(gpu)
    out = torch.full((int(q_off[-1]),), -7, dtype=torch.int32, device=gpu)
    cnt = torch.full((3,), -7, dtype=torch.int32, device=gpu)
    m.search_by_projection_batch_device(PROJ_FRAME_MAPPOINTS, fb, T(np.concatenate(ds)),
                                        T(np.concatenate(qs)), torch.from_numpy(q_off).to(gpu),
                                        out, cnt, orb_dist=64)
    with pytest.raises(OrbxError):
        m.sync()
    out, cnt = out.cpu().numpy(), cnt.cpu().numpy()
    assert cnt[2] == 0 and (out[q_off[2]:] == -1).all()
    for j in range(2):
        n_o, m_o = om.search_by_projection(PROJ_FRAME_MAPPOINTS, frames[j], qs[j], ds[j],
                                           None, None, orb_dist=64, nnratio=0.8)
        assert cnt[j] == n_o
        np.testing.assert_array_equal(out[q_off[j]:q_off[j + 1]], m_o)


def test_distinctive_descriptors(oracle_mod, orbx_lib, gpu):
    from oracle import matcher as om
    from test_oracle_match import _distinctive_case
    for seed, npts, maxn in [(0, 500, 40), (1, 40, 256)]:
        desc, off = _distinctive_case(seed, npts, maxn)
        m = _matcher(0.6, True)
        np.testing.assert_array_equal(m.compute_distinctive_descriptors(desc, off),
                                      om.distinctive_descriptors(desc, off))
