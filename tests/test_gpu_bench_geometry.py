"""Parity at the benchmarked geometries: every workload bench.py times, at exactly the size and
launch geometry it times, built by bench.py's own input builders.

* C2 (the headline, configs[1]): 512 KITTI stereo pairs per call, resident in the pyramid's
  level-0 slots as bench.py times them (the copying tensor path is covered by
  test_gpu_extract.py and test_resident_equals_tensor_path below).  At 1024 images every
  pyramid level walks 64-row strips and k_stereo runs one workgroup per pair (asserted through
  orbx_extractor_launch_info); a single image runs 8-row strips and split stereo.  Every slot
  must equal its single-image run, and 16 slots must equal the CPU restatement bit for bit
  (ORBextractor.cc:1065-1154, Frame.cc:496-686).
* C3 (configs[2]): 256 EuRoC frames through MonoTrackBatch with a 2000-MapPoint 3-D local map
  per frame, projected on the device (isInFrustum + PredictScale, Frame.cc:285-349,
  MapPoint.cc:430-444) inside the step, every slot's queries, in-view count and matches
  against the restatement (ORBmatcher.cc:41-136).
* C4 (configs[3]): the 10k-keyframe relocalisation database, 512 sampled keyframes (the 10
  planted true ones among them) against SearchByBoW(KF, F) restated (ORBmatcher.cc:182-319).
* C4 pure brute force (bench.py --workload bf): one 1000-descriptor query frame against the
  10^7-row database, whole and in 3 / 8 shards (global row numbers, merge in shard order);
  every planted query finds its row, and 64 queries equal the restated loop over all 10^7
  rows (ORBmatcher.cc:232-256).
* C5 (configs[4]): all 512 SearchForTriangulation jobs against the restatement
  (ORBmatcher.cc:702-872).
"""
import numpy as np
import pytest

import bench
from helpers import assert_bytes_equal, assert_f32_bits_equal, assert_kps_equal

pytestmark = pytest.mark.gpu


def test_c2_stereo_b512(oracle_mod, orbx_lib, gpu):
    import torch
    import my_orb_slam2_amd as m
    B = 512
    Lh, Rh, _, n_distinct = bench.stereo_inputs(0, B, 32)
    assert n_distinct == B
    Ls, Rs = torch.from_numpy(Lh).to(gpu), torch.from_numpy(Rh).to(gpu)
    mb = float(np.float32(bench.MBF) / np.float32(bench.FX))
    sb = m.StereoBatch(B, bench.NFEAT, 1.2, 8, 20, 7)
    # the timed path: the pairs sit in the pyramid's level-0 slots (bench.py --input resident)
    Lv, Rv = sb.input_views(bench.W, bench.H)
    Lv.copy_(Ls)
    Rv.copy_(Rs)
    uR, dep, nv = sb.run_resident(bench.MBF, mb)
    torch.cuda.synchronize()
    rows, split = sb.ext.launch_info(2 * B)
    assert (rows == 64).all() and split == 1, (rows, split)   # the timed geometry
    nkp, kps, desc = sb.fetch("left")
    nkpr, kpsr, descr = sb.fetch("right")
    uRh, deph, nvh = uR.cpu().numpy(), dep.cpu().numpy(), nv.cpu().numpy()
    gl = m.ORBextractor(bench.NFEAT, 1.2, 8, 20, 7)
    gr = m.ORBextractor(bench.NFEAT, 1.2, 8, 20, 7)
    gl(Lh[0])
    rows1, split1 = gl.launch_info(1)
    assert (rows1 == 8).all(), rows1                           # the single-image geometry
    for i in range(B):
        k1, d1 = gl(Lh[i])
        k2, d2 = gr(Rh[i])
        assert nkp[i] == len(k1) and nkpr[i] == len(k2), f"slot {i} keypoint counts"
        assert_kps_equal(kps[i, :nkp[i]], k1, f"slot {i} left")
        assert_bytes_equal(desc[i, :nkp[i]], d1, f"slot {i} left desc")
        assert_kps_equal(kpsr[i, :nkpr[i]], k2, f"slot {i} right")
        assert_bytes_equal(descr[i, :nkpr[i]], d2, f"slot {i} right desc")
        u1, z1, n1 = m.compute_stereo_matches(gl, gr, bench.MBF, mb)
        assert_f32_bits_equal(uRh[i, :nkp[i]], u1, f"slot {i} uRight")
        assert_f32_bits_equal(deph[i, :nkp[i]], z1, f"slot {i} depth")
        assert nvh[i] == n1, f"slot {i} valid stereo matches"
    assert nvh.min() > 100
    # 16 slots spread over the batch (both roll offsets and base pairs vary) vs the oracle
    for i in np.linspace(0, B - 1, 16).astype(int):
        ol = oracle_mod.OracleExtractor(bench.NFEAT, 1.2, 8, 20, 7)
        orr = oracle_mod.OracleExtractor(bench.NFEAT, 1.2, 8, 20, 7)
        k_o, d_o = ol(Lh[i])
        kr_o, dr_o = orr(Rh[i])
        assert_kps_equal(kps[i, :nkp[i]], k_o, f"slot {i} left vs oracle")
        assert_bytes_equal(desc[i, :nkp[i]], d_o, f"slot {i} left desc vs oracle")
        assert_kps_equal(kpsr[i, :nkpr[i]], kr_o, f"slot {i} right vs oracle")
        assert_bytes_equal(descr[i, :nkpr[i]], dr_o, f"slot {i} right desc vs oracle")
        u_o, z_o, n_o = oracle_mod.stereo_match(ol, orr, len(k_o), bench.MBF, mb)
        assert_f32_bits_equal(uRh[i, :nkp[i]], u_o, f"slot {i} uRight vs oracle")
        assert_f32_bits_equal(deph[i, :nkp[i]], z_o, f"slot {i} depth vs oracle")
        assert nvh[i] == n_o


def test_c2_timed_schedule_b512(oracle_mod, orbx_lib, gpu):
    """The headline's exact timed configuration (bench.headline_handles, as bench.py builds
    it): two StereoBatch handles of 512 pairs alternating steps on two torch streams, each
    extraction with the side branch 3,3,1, six steps.  Every slot of both handles equals the
    single-handle one-stream run (overlap 0) of the same pairs, and 16 slots equal the CPU
    restatement (ORBextractor.cc:1065-1154, Frame.cc:496-686).  The inputs are the headline's:
    512 independent generated scenes (bench.py's default --distinct)."""
    import torch
    import my_orb_slam2_amd as m
    B = 512
    Lh, Rh, pairs, n_distinct = bench.stereo_inputs(0, B, B)
    assert len(pairs) == B and n_distinct == B
    Ls, Rs = torch.from_numpy(Lh).to(gpu), torch.from_numpy(Rh).to(gpu)
    mb = float(np.float32(bench.MBF) / np.float32(bench.FX))
    sbs, sts, run_on, run_step, overlap = bench.headline_handles(
        torch, m, gpu, 0, B, Ls, Rs, 2, "3,3,1", True, mb)
    assert overlap == (3, 3, 1)
    for i in range(6):
        run_step(i)
    torch.cuda.synchronize()
    got = [bench.stereo_digests(h) for h in sbs]
    # the reference schedule: one handle, every kernel in sequence on one stream
    sbs[0].ext.set_overlap(0)
    run_on(sbs[0], sts[0])
    torch.cuda.synchronize()
    ref = bench.stereo_digests(sbs[0])
    for k in range(2):
        bad = [i for i in range(B) if got[k][i] != ref[i]]
        assert not bad, f"handle {k}: slots {bad[:8]} differ from the one-stream run"
    v = bench.verification(got, ref, B)
    assert v["verified"] and v["mismatched_slots"] == 0
    for i in np.linspace(0, B - 1, 16).astype(int):
        ol = oracle_mod.OracleExtractor(bench.NFEAT, 1.2, 8, 20, 7)
        orr = oracle_mod.OracleExtractor(bench.NFEAT, 1.2, 8, 20, 7)
        k_o, d_o = ol(Lh[i])
        kr_o, dr_o = orr(Rh[i])
        u_o, z_o, n_o = oracle_mod.stereo_match(ol, orr, len(k_o), bench.MBF, mb)
        assert bench.slot_digest(k_o, d_o, kr_o, dr_o, u_o, z_o, n_o) == got[1][i], \
            f"slot {i} differs from the oracle"


def test_c3_euroc_b256(oracle_mod, orbx_lib, gpu):
    import torch
    from oracle import matcher as om
    from my_orb_slam2_amd import synth
    from my_orb_slam2_amd.features import (PROJ_FRAME_MAPPOINTS, PROJ_QUERY_DTYPE, FeatureSet,
                                           assign_features_to_grid)
    from my_orb_slam2_amd.tracking import MonoTrackBatch
    B, P, NQ = 256, 32, 2000
    K4, dist = synth.EUROC_CAM
    frames, idx = bench.euroc_frames(0, B, P)
    d_imgs = torch.from_numpy(np.stack([frames[i] for i in idx])).to(gpu)
    mt = MonoTrackBatch(B, bench.EUROC_W, bench.EUROC_H, K4, dist, bench.EUROC_NFEAT,
                        device=gpu.index or 0)
    rows, _ = mt.ext.launch_info(B)
    mt.frames(d_imgs)
    nkp, ku, desc = mt.fetch_undistorted()
    per = bench.euroc_local_maps(idx, nkp, ku, desc, NQ, mt.kp_cap, mt.bounds)
    inp = bench.euroc_device_inputs(torch, gpu, per, idx)
    q_off = inp["q_off_h"]
    out = torch.full((int(q_off[-1]),), -7, dtype=torch.int32, device=gpu)
    cnt = torch.full((B,), -7, dtype=torch.int32, device=gpu)
    # the timed step: frames, the local maps' projection (isInFrustum + PredictScale), search
    mt(d_imgs, inp["desc"], inp["q"], inp["q_off"], out, cnt, inp["claimed"],
       local_map=(inp["frames"], inp["mps"], inp["max_mps"], inp["skip"], inp["nvis"], 1.0))
    mt.matcher.sync()
    out, cnt = out.cpu().numpy(), cnt.cpu().numpy()
    qg = inp["q"].cpu().numpy().reshape(-1, 32)
    nvis = inp["nvis"].cpu().numpy()
    _, kraw, _ = mt.ext.batch_fetch(0, B)
    ref = {}
    for p in range(P):
        ox = oracle_mod.OracleExtractor(bench.EUROC_NFEAT, 1.2, 8, 20, 7)
        k_o, d_o = ox(frames[p])
        un = om.undistort_keypoints(k_o, K4, dist)
        ku_o = k_o.copy()
        ku_o["x"], ku_o["y"] = un[:, 0], un[:, 1]
        g = assign_features_to_grid(ku_o, *mt.bounds)
        pose, mps, d, skip, cl = per[p]
        qb, nv_o = om.is_in_frustum(pose, mps, skip, 0.5, 1.0)
        ref[p] = (k_o, d_o, ku_o, qb.reshape(-1, 32), nv_o, om.search_by_projection(
            PROJ_FRAME_MAPPOINTS, FeatureSet(ku_o, d_o, None, None, g),
            qb.view(PROJ_QUERY_DTYPE), d, cl[:len(k_o)], None, nnratio=0.8))
    for b, p in enumerate(idx):
        k_o, d_o, ku_o, q_o, nv_o, (n_o, m_o) = ref[p]
        assert nvis[b] == nv_o, f"frame {b} MapPoints in view"
        bad = np.nonzero((qg[q_off[b]:q_off[b + 1]] != q_o).any(1))[0]
        assert bad.size == 0, f"frame {b}: projections of MapPoints {bad[:8]} differ"
        n = int(nkp[b])
        assert_kps_equal(kraw[b, :n], k_o, f"frame {b} keypoints")
        assert_bytes_equal(desc[b, :n], d_o, f"frame {b} descriptors")
        np.testing.assert_array_equal(ku[b, :n]["x"].view(np.int32), ku_o["x"].view(np.int32))
        np.testing.assert_array_equal(ku[b, :n]["y"].view(np.int32), ku_o["y"].view(np.int32))
        assert cnt[b] == n_o, f"frame {b} match count"
        np.testing.assert_array_equal(out[q_off[b]:q_off[b + 1]], m_o, f"frame {b} matches")
    assert cnt.min() > 300
    assert rows.max() == 64   # the large levels walk full-height strips at 256 frames


def test_c4_relocalisation_10k(oracle_mod, orbx_lib, gpu):
    import torch
    from oracle import matcher as om
    from my_orb_slam2_amd import ORBmatcher
    from my_orb_slam2_amd._lib import KEYPOINT_DTYPE
    from my_orb_slam2_amd.features import FeatureSet, FeatureSetC, feature_vector
    K, F = 10000, 1000
    db, keep, _ = bench._reloc_db(torch, gpu, 0, K, F)
    qdesc, qkeys, true_kfs = bench._reloc_query(torch, gpu, K, F)
    qn_off = torch.tensor([0, F], dtype=torch.int32, device=gpu)
    q_node = torch.zeros(1, dtype=torch.int32, device=gpu)
    q_feat = torch.arange(F, dtype=torch.int32, device=gpu)
    fc = FeatureSetC()
    fc.n, fc.keys, fc.desc = F, qkeys.data_ptr(), qdesc.data_ptr()
    fc.n_nodes, fc.node_id, fc.node_off, fc.node_feat = (1, q_node.data_ptr(), qn_off.data_ptr(),
                                                        q_feat.data_ptr())
    mt = ORBmatcher(0.75, True)
    out = torch.full((K, F), -7, dtype=torch.int32, device=gpu)
    cnt = torch.full((K,), -7, dtype=torch.int32, device=gpu)
    mt.search_by_bow_kf_frame_batch_device(db, fc, out, cnt)
    mt.sync()
    cnt_h = cnt.cpu().numpy()
    assert (cnt_h[true_kfs.numpy()] >= 15).all()

    def fs(d, k):
        kp = np.zeros(len(d), KEYPOINT_DTYPE)
        kp["angle"] = k[:, 3]
        return FeatureSet(kp, d, None, feature_vector(np.zeros(len(d))), None)
    frame = fs(qdesc.cpu().numpy(), qkeys.cpu().numpy())
    desc, keys, flag = keep[0], keep[1], keep[2]
    rng = np.random.default_rng(0)
    sample = np.unique(np.concatenate([true_kfs.numpy(), rng.choice(K, 502, replace=False)]))
    assert len(sample) >= 500
    for k in sample:
        sl = slice(int(k) * F, (int(k) + 1) * F)
        n_o, m_o = om.search_by_bow_kf_frame(fs(desc[sl].cpu().numpy(), keys[sl].cpu().numpy()),
                                             flag[sl].cpu().numpy(), frame, 0.75, True)
        assert cnt_h[k] == n_o, f"keyframe {k}"
        np.testing.assert_array_equal(out[k].cpu().numpy(), m_o, f"keyframe {k}")


def test_c4_bf_10m(orbx_lib, gpu):
    import torch
    from oracle import matcher as om
    from my_orb_slam2_amd import ORBmatcher
    from my_orb_slam2_amd.distributed import merge_top2, shard_range
    ndb = 10_000_000
    db = np.empty((ndb, 32), np.uint8)
    for b0 in range(0, ndb, 1 << 20):
        b1 = min(b0 + (1 << 20), ndb)
        db[b0:b1] = bench.bf_rows(b0, b1)
    q, ids, rows = bench.bf_query(ndb)
    nq = len(q)
    ddb, dq = torch.from_numpy(db).to(gpu), torch.from_numpy(q).to(gpu)
    m = ORBmatcher(0.75, True)

    def run(world):
        parts = []
        for r in range(world):
            r0, r1 = shard_range(ndb, r, world)
            out = [torch.full((nq,), -7, dtype=torch.int32, device=gpu) for _ in range(3)]
            m.hamming_bf_top2_device(dq, nq, ddb[r0:], r1 - r0, *out, idx_base=r0)
            parts.append(tuple(out))
        torch.cuda.synchronize(gpu)
        return [t.cpu().numpy() for t in merge_top2(parts)] if world > 1 else \
            [t.cpu().numpy() for t in parts[0]]
    bi, bd, sd = run(1)
    np.testing.assert_array_equal(bi[ids], rows)          # every planted row found
    assert bd[ids].max() <= 40 and (bd >= 0).all() and (sd >= bd).all()
    for world in (3, 8):
        for g, w in zip(run(world), (bi, bd, sd)):
            np.testing.assert_array_equal(g, w)
    sample = np.unique(np.concatenate([ids[:16], np.linspace(0, nq - 1, 48).astype(int)]))
    want = om.bf_top2(q[sample], db)
    for g, w in zip((bi[sample], bd[sample], sd[sample]), want):
        np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("node_order", [False, True], ids=["gather", "node_order"])
def test_c5_triangulation_512(oracle_mod, orbx_lib, gpu, node_order):
    """All 512 C5 jobs vs the restatement, with the database's features gathered by index and
    with its node-order copies (orbx_kf_db_node_order: the bench's layout)."""
    import torch
    from oracle import matcher as om
    from my_orb_slam2_amd import ORBmatcher, synth
    from my_orb_slam2_amd.matcher import DeviceKfDb
    J = 512
    kfs, flags, F12, epi = bench.triangulation_jobs(0, J)
    db = DeviceKfDb(kfs, flags, gpu)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    n1 = np.array([kfs[2 * i].n for i in range(J)], np.int32)
    job_off = np.concatenate([[0], np.cumsum(n1)]).astype(np.int32)
    s, s2, _ = synth.scale_tables()
    mt = ORBmatcher(0.6, False)
    if node_order:
        db.node_order(mt)
        torch.cuda.synchronize()
    out = torch.full((int(job_off[-1]),), -7, dtype=torch.int32, device=gpu)
    cnt = torch.full((J,), -7, dtype=torch.int32, device=gpu)
    mt.search_for_triangulation_batch_device(db.c, T(np.arange(J, dtype=np.int32) * 2),
                                             T(np.arange(J, dtype=np.int32) * 2 + 1),
                                             T(np.array(F12, np.float32)),
                                             T(np.array(epi, np.float32)), s2, s, T(job_off), out,
                                             cnt)
    mt.sync()
    out, cnt = out.cpu().numpy(), cnt.cpu().numpy()
    for j in range(J):
        n_o, p_o = om.search_for_triangulation(kfs[2 * j], flags[2 * j], kfs[2 * j + 1],
                                               flags[2 * j + 1], F12[j].reshape(3, 3), epi[j], s2,
                                               s, False, False)
        seg = out[job_off[j]:job_off[j + 1]]
        idx1 = np.nonzero(seg >= 0)[0]
        assert cnt[j] == n_o, f"job {j}"
        np.testing.assert_array_equal(np.stack([idx1, seg[idx1]], 1), p_o, f"job {j}")
    assert cnt.min() > 0


def test_resident_equals_tensor_path(orbx_lib, gpu):
    """The level-0-in-place path (orbx_stereo_frames_resident) and the copying path
    (orbx_stereo_frames_device, strided caller tensor) give the same bits at 96 pairs."""
    import torch
    import my_orb_slam2_amd as m
    B = 96
    Lh, Rh, _, _ = bench.stereo_inputs(3, B, 8)
    Ls, Rs = torch.from_numpy(Lh).to(gpu), torch.from_numpy(Rh).to(gpu)
    mb = float(np.float32(bench.MBF) / np.float32(bench.FX))
    a, b = m.StereoBatch(B, bench.NFEAT), m.StereoBatch(B, bench.NFEAT)
    ua, da, na = (t.clone() for t in a(Ls, Rs, bench.MBF, mb))
    Lv, Rv = b.input_views(bench.W, bench.H)
    Lv.copy_(Ls)
    Rv.copy_(Rs)
    ub, db, nb = b.run_resident(bench.MBF, mb)
    torch.cuda.synchronize()
    assert torch.equal(na, nb)
    nkp = a.fetch("left")[0]
    ua, ub, da, db = (t.cpu().numpy() for t in (ua, ub, da, db))
    for i in range(B):   # slots past a pair's keypoint count are not written
        assert_f32_bits_equal(ub[i, :nkp[i]], ua[i, :nkp[i]], f"pair {i} uRight")
        assert_f32_bits_equal(db[i, :nkp[i]], da[i, :nkp[i]], f"pair {i} depth")
    for side in ("left", "right"):
        ka, kb = a.fetch(side), b.fetch(side)
        assert np.array_equal(ka[0], kb[0])
        for i in range(B):
            n = ka[0][i]
            assert_kps_equal(kb[1][i, :n], ka[1][i, :n], f"{side} {i}")
            assert_bytes_equal(kb[2][i, :n], ka[2][i, :n], f"{side} {i} desc")
        # the level-0 slots hold the inputs untouched by the extraction
    assert torch.equal(Lv, Ls) and torch.equal(Rv, Rs)
