"""CPU (gloo, world_size 2) tests of the multi-GPU plumbing: shard ranges, query broadcast and
the count all-gather used by the sharded relocalisation / triangulation workloads."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from my_orb_slam2_amd.distributed import (CandidateOverflow, all_gather_counts, broadcast_query,
                                          candidate_block, gather_candidate_matches, gather_rows,
                                          merge_candidate_blocks, relocalisation_candidates,
                                          shard_range)


@pytest.mark.parametrize("n,world", [(10000, 8), (7, 3), (3, 4), (0, 2), (512, 8)])
def test_shard_range_partitions(n, world):
    spans = [shard_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (b0, e0), (b1, e1) in zip(spans, spans[1:]):
        assert e0 == b1
    sizes = [e - b for b, e in spans]
    assert max(sizes) - min(sizes) <= 1


def _worker(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        desc = torch.zeros(5, 32, dtype=torch.uint8)
        if rank == 0:
            desc[:] = torch.arange(160, dtype=torch.uint8).reshape(5, 32)
        broadcast_query([desc])
        b, e = shard_range(n_total, rank, world)
        # each rank "matches" its shard: count = global keyframe id % 20
        local = torch.arange(b, e, dtype=torch.int32) % 20
        allc = all_gather_counts(local, n_total, world)
        # per-keyframe match rows: feature f of keyframe k matched to (k * 7 + f) % 11, or -1
        F = 6
        kf = torch.arange(b, e, dtype=torch.int32)[:, None]
        feat = torch.arange(F, dtype=torch.int32)[None, :]
        rows = torch.where(feat < 4, (kf * 7 + feat) % 11, torch.full_like(kf * feat, -1))
        everything = gather_rows(rows, n_total, world)
        cand = gather_candidate_matches(rows, allc, n_total, world)
        # a block of 1 candidate per rank overflows (each rank owns 4-5 candidates): both ranks
        # read the headers and gather again with room for all of them
        cand_small = gather_candidate_matches(rows, allc, n_total, world, cap=1)
        q.put((rank, desc.sum().item(), allc.numpy().tolist(), everything.numpy().tolist(),
               [(k, np.asarray(m).tolist()) for k, m in cand],
               [(k, np.asarray(m).tolist()) for k, m in cand_small]))
    finally:
        dist.destroy_process_group()


def test_gloo_broadcast_and_gather():
    world, n_total = 2, 37
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    expect = (np.arange(n_total) % 20).tolist()
    F = 6
    rows = [[(k * 7 + f) % 11 if f < 4 else -1 for f in range(F)] for k in range(n_total)]
    want_cand = [(k, rows[k]) for k in range(n_total) if k % 20 >= 15]
    for rank, s, allc, everything, cand, cand_small in res:
        assert s == int(np.arange(160).sum())
        assert allc == expect
        assert everything == rows
        assert cand == want_cand
        assert cand_small == want_cand
    cand = relocalisation_candidates(np.array(expect))
    np.testing.assert_array_equal(cand, [i for i in range(n_total) if i % 20 >= 15])


def test_candidate_block_reports_overflow():
    """A rank with more candidates than its block holds is reported, not truncated (ADVICE r3:
    Tracking::Relocalization keeps every keyframe with >= 15 matches, Tracking.cc:1487)."""
    n, F = 40, 3
    counts = torch.tensor([20 if k % 3 == 0 else 3 for k in range(n)], dtype=torch.int32)
    rows = torch.arange(n * F, dtype=torch.int32).reshape(n, F)
    want = [k for k in range(n) if k % 3 == 0]            # 14 candidates
    blk = candidate_block(rows, counts, 100, cap=len(want))
    got = merge_candidate_blocks([blk])
    assert [k for k, _ in got] == [100 + k for k in want]
    for k, m in got:
        np.testing.assert_array_equal(m, rows[k - 100].numpy())
    with pytest.raises(CandidateOverflow) as ei:
        merge_candidate_blocks([candidate_block(rows, counts, 100, cap=5), blk])
    assert ei.value.needed == len(want) and ei.value.cap == 5
    # no candidate at all: an empty list, header count 0
    assert merge_candidate_blocks([candidate_block(rows, counts * 0, 0, cap=4)]) == []
