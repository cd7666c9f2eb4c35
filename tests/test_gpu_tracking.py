"""GPU parity of the batched mono tracking front-end (my_orb_slam2_amd/tracking.py): EuRoC
752x480 frames through extraction, undistortion, grid and SearchLocalPoints' projection
search, against the CPU restatement stage by stage (bit-exact keypoints, undistorted
coordinates, grid CSR and match indices)."""
import numpy as np
import pytest

from my_orb_slam2_amd import synth
from my_orb_slam2_amd.features import FeatureSet, assign_features_to_grid

pytestmark = pytest.mark.gpu

W, H = 752, 480


def test_mono_track_batch(oracle_mod, orbx_lib, gpu):
    import torch
    import oracle
    from oracle import matcher as om
    from my_orb_slam2_amd.features import PROJ_FRAME_MAPPOINTS
    from my_orb_slam2_amd.tracking import MonoTrackBatch
    K4, dist = synth.EUROC_CAM
    B = 6
    imgs = np.stack([synth.frame(500 + i, W, H) for i in range(B)])
    imgs[3] = 0   # a frame without features
    mt = MonoTrackBatch(B, W, H, K4, dist, device=gpu.index or 0)
    d_imgs = torch.from_numpy(imgs).to(gpu)
    mt.frames(d_imgs)
    nkp, ku, desc = mt.fetch_undistorted()
    assert nkp[3] == 0 and (nkp[[0, 1, 2, 4, 5]] > 900).all()

    # extraction of one frame against the restatement
    ox = oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
    k_o, d_o = ox(imgs[0])
    _, kraw, _ = mt.ext.batch_fetch(0, 1)
    np.testing.assert_array_equal(kraw[0, :nkp[0]].view(np.uint8), k_o.view(np.uint8))
    np.testing.assert_array_equal(desc[0, :nkp[0]], d_o)

    qs, ds, cls, refs = [], [], [], []
    bounds = mt.bounds
    _, _, isg = synth.scale_tables()
    for j in range(B):
        n = int(nkp[j])
        _, kr, _ = mt.ext.batch_fetch(j, 1)
        un = om.undistort_keypoints(kr[0, :n], K4, dist) if n else np.zeros((0, 2), np.float32)
        np.testing.assert_array_equal(ku[j, :n]["x"].view(np.int32), un[:, 0].view(np.int32))
        np.testing.assert_array_equal(ku[j, :n]["y"].view(np.int32), un[:, 1].view(np.int32))
        g = assign_features_to_grid(ku[j, :n], *bounds)
        np.testing.assert_array_equal(mt.grid_off[j].cpu().numpy(), g.off)
        np.testing.assert_array_equal(mt.grid_feat[j, :len(g.feat)].cpu().numpy(), g.feat)
        q, d = synth.local_map_queries(j, ku[j, :n], desc[j, :n], 1500 + 100 * j, W, H)
        cl = np.zeros(mt.kp_cap, np.uint8)
        cl[:n] = np.random.default_rng(j).random(n) < 0.2
        fs = FeatureSet(ku[j, :n].copy(), desc[j, :n].copy(), None, None, g)
        refs.append(om.search_by_projection(PROJ_FRAME_MAPPOINTS, fs, q, d, cl[:n], None,
                                            nnratio=0.8))
        qs.append(q)
        ds.append(d)
        cls.append(cl)
    q_off = np.concatenate([[0], np.cumsum([len(q) for q in qs])]).astype(np.int32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(gpu)
    out = torch.full((int(q_off[-1]),), -7, dtype=torch.int32, device=gpu)
    cnt = torch.full((B,), -7, dtype=torch.int32, device=gpu)
    # the whole pipeline once more in one call (extraction repeated: same results)
    mt(d_imgs, T(np.concatenate(ds)), T(np.concatenate(qs)), torch.from_numpy(q_off).to(gpu),
       out, cnt, T(np.concatenate(cls)))
    mt.matcher.sync()
    out, cnt = out.cpu().numpy(), cnt.cpu().numpy()
    for j, (n_o, m_o) in enumerate(refs):
        assert cnt[j] == n_o, j
        np.testing.assert_array_equal(out[q_off[j]:q_off[j + 1]], m_o)
    assert cnt[[0, 1, 2, 4, 5]].min() > 300
