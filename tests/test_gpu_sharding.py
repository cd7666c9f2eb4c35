"""Sharding correctness on one device: the relocalisation database (C4) and the
triangulation jobs (C5) split into N shard_range slices, each slice run as its own rank would
run it, the per-rank buffers merged with the same pure functions the collectives use
(my_orb_slam2_amd/distributed.py: pad_shard / merge_shards / candidate_block /
merge_candidate_blocks).  The merged result must equal the unsharded run, for N = 2, 3, 8."""
import numpy as np
import pytest

import bench
from my_orb_slam2_amd.distributed import (candidate_block, merge_candidate_blocks, merge_shards,
                                          pad_shard, shard_range)

pytestmark = pytest.mark.gpu


def _reloc(torch, gpu, k0, k1, F, query):
    from my_orb_slam2_amd import ORBmatcher
    from my_orb_slam2_amd.features import FeatureSetC
    db, keep, _ = bench._reloc_db(torch, gpu, k0, k1, F)
    qdesc, qkeys = query
    qn_off = torch.tensor([0, F], dtype=torch.int32, device=gpu)
    q_node = torch.zeros(1, dtype=torch.int32, device=gpu)
    q_feat = torch.arange(F, dtype=torch.int32, device=gpu)
    fc = FeatureSetC()
    fc.n, fc.keys, fc.desc = F, qkeys.data_ptr(), qdesc.data_ptr()
    fc.n_nodes, fc.node_id, fc.node_off, fc.node_feat = (1, q_node.data_ptr(), qn_off.data_ptr(),
                                                        q_feat.data_ptr())
    m = ORBmatcher(0.75, True)
    out = torch.full((k1 - k0, F), -7, dtype=torch.int32, device=gpu)
    cnt = torch.full((k1 - k0,), -7, dtype=torch.int32, device=gpu)
    m.search_by_bow_kf_frame_batch_device(db, fc, out, cnt)
    m.sync()
    del keep
    return out, cnt


def test_relocalisation_shards_merge(orbx_lib, gpu):
    import torch
    K, F = 1200, 1000
    qdesc, qkeys, true_kfs = bench._reloc_query(torch, gpu, K, F)
    full_out, full_cnt = _reloc(torch, gpu, 0, K, F, (qdesc, qkeys))
    full_cand = [(int(k), full_out[k].cpu().numpy())
                 for k in np.nonzero(full_cnt.cpu().numpy() >= 15)[0]]
    assert {k for k, _ in full_cand} >= set(true_kfs.numpy().tolist())
    for world in (2, 3, 8):
        counts, rows, blocks = [], [], []
        for r in range(world):
            k0, k1 = shard_range(K, r, world)
            out, cnt = _reloc(torch, gpu, k0, k1, F, (qdesc, qkeys))
            counts.append(pad_shard(cnt, K, world))
            rows.append(pad_shard(out, K, world))
            blocks.append(candidate_block(out, cnt, k0))
        assert torch.equal(merge_shards(counts, K, world), full_cnt), world
        assert torch.equal(merge_shards(rows, K, world), full_out), world
        cand = merge_candidate_blocks(blocks)
        assert [k for k, _ in cand] == [k for k, _ in full_cand], world
        for (k, m), (k2, m2) in zip(cand, full_cand):
            np.testing.assert_array_equal(m, m2)


def test_triangulation_shards_merge(orbx_lib, gpu):
    import torch
    from my_orb_slam2_amd import ORBmatcher, synth
    from my_orb_slam2_amd.matcher import DeviceKfDb
    J = 512
    s, s2, _ = synth.scale_tables()
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    cache = {}

    def run(j0, j1):
        kfs, flags, F12, epi = [], [], [], []
        for j in range(j0, j1):
            if j not in cache:
                cache[j] = bench.triangulation_jobs(j, j + 1)
            a, b, c, d = cache[j]
            kfs += a
            flags += b
            F12 += c
            epi += d
        db = DeviceKfDb(kfs, flags, gpu)
        nj = j1 - j0
        n1 = np.array([kfs[2 * i].n for i in range(nj)], np.int32)
        job_off = np.concatenate([[0], np.cumsum(n1)]).astype(np.int32)
        m = ORBmatcher(0.6, False)
        out = torch.full((int(job_off[-1]),), -7, dtype=torch.int32, device=gpu)
        cnt = torch.full((nj,), -7, dtype=torch.int32, device=gpu)
        m.search_for_triangulation_batch_device(db.c, T(np.arange(nj, dtype=np.int32) * 2),
                                                T(np.arange(nj, dtype=np.int32) * 2 + 1),
                                                T(np.array(F12, np.float32)),
                                                T(np.array(epi, np.float32)), s2, s, T(job_off),
                                                out, cnt)
        m.sync()
        return out.view(nj, -1), cnt

    full_rows, full_cnt = run(0, J)
    for world in (2, 3, 8):
        rows, counts = [], []
        for r in range(world):
            j0, j1 = shard_range(J, r, world)
            o, c = run(j0, j1)
            rows.append(pad_shard(o, J, world))
            counts.append(pad_shard(c, J, world))
        assert torch.equal(merge_shards(counts, J, world), full_cnt), world
        assert torch.equal(merge_shards(rows, J, world), full_rows), world
    assert int(full_cnt.min()) > 0
