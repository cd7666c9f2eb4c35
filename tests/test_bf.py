"""Brute-force Hamming top-2 (orbx_hamming_bf_top2, SURVEY §8(b) / §8(e) C4 pure BF).

The oracle (oracle/orb_matcher_oracle.cpp: oracle_bf_top2) is the best / second loop of
src/ORBmatcher.cc:232-256 over every database row; here it is checked against an independent
numpy restatement, the shard merge (distributed.merge_top2) against the whole-database
result, the gloo all-gather path at world size 2, and the GPU kernels against the oracle."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle.matcher as om
from my_orb_slam2_amd.distributed import gather_top2, merge_top2, shard_range


def bf_database(seed, nq, ndb, planted=True):
    """Random descriptors with planted structure: exact copies of queries (distance 0) placed
    twice at distant rows (a tie the first row must win), near copies (a few bits flipped), and
    complements of queries (distance 256, which the loop never takes as best)."""
    rng = np.random.default_rng(seed)
    q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    db = rng.integers(0, 256, (ndb, 32), dtype=np.uint8)
    if planted and ndb >= 4 and nq:
        for i in range(min(nq, ndb // 4)):
            kind = i % 4
            r = int(rng.integers(0, ndb))
            if kind == 0:                        # two exact copies: the first row must win
                r2 = int(rng.integers(0, ndb))
                db[r] = q[i]
                db[r2] = q[i]
            elif kind == 1:                      # near copy
                db[r] = q[i]
                for b in rng.choice(256, int(rng.integers(1, 40)), replace=False):
                    db[r, b // 8] ^= np.uint8(1 << (b % 8))
            elif kind == 2:                      # complement: distance 256
                db[r] = ~q[i]
    return q, db


def numpy_top2(q, db):
    """Independent restatement: the full distance matrix, then best = first argmin below 256,
    second = the second least of the multiset {256, 256} ∪ row distances."""
    nq = len(q)
    if len(db) == 0:
        return (np.full(nq, -1, np.int32), np.full(nq, 256, np.int32), np.full(nq, 256, np.int32))
    d = np.unpackbits(q[:, None, :] ^ db[None, :, :], axis=2).sum(axis=2).astype(np.int32)
    ext = np.concatenate([d, np.full((nq, 2), 256, np.int32)], axis=1)
    srt = np.sort(ext, axis=1)
    b1, b2 = srt[:, 0], srt[:, 1]
    idx = np.where(b1 < 256, np.argmin(d, axis=1), -1).astype(np.int32)
    return idx, b1.astype(np.int32), b2.astype(np.int32)


@pytest.mark.parametrize("seed,nq,ndb", [(0, 40, 3000), (1, 7, 1), (2, 5, 0), (3, 64, 2),
                                         (4, 33, 517)])
def test_oracle_matches_numpy(seed, nq, ndb):
    q, db = bf_database(seed, nq, ndb)
    got = om.bf_top2(q, db)
    want = numpy_top2(q, db)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


def test_oracle_ties_and_complements():
    q = np.zeros((3, 32), np.uint8)
    q[1] = 0xFF
    q[2, 0] = 1
    db = np.stack([np.full(32, 0xFF, np.uint8), np.zeros(32, np.uint8), np.zeros(32, np.uint8)])
    bi, bd, sd = om.bf_top2(q, db)
    # query 0: row 0 is at 256 (never the best), rows 1 and 2 tie at 0: row 1, second 0
    assert (bi[0], bd[0], sd[0]) == (1, 0, 0)
    # query 1: row 0 at 0, rows 1-2 at 256: second stays 256
    assert (bi[1], bd[1], sd[1]) == (0, 0, 256)
    assert (bi[2], bd[2], sd[2]) == (1, 1, 1)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_shard_merge_equals_whole(world):
    q, db = bf_database(5, 50, 4001)
    whole = om.bf_top2(q, db)
    parts = [om.bf_top2(q, db, *shard_range(len(db), r, world)) for r in range(world)]
    merged = merge_top2(parts)
    for g, w in zip(merged, whole):
        np.testing.assert_array_equal(np.asarray(g), w)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q, db = bf_database(6, 30, 1999)
        r0, r1 = shard_range(len(db), rank, world)
        bi, bd, sd = (torch.from_numpy(np.asarray(x, np.int32)) for x in om.bf_top2(q, db, r0, r1))
        m = gather_top2(bi, bd, sd, world)
        out.put((rank, [t.numpy().tolist() for t in m]))
    finally:
        dist.destroy_process_group()


def test_gloo_gather_top2():
    world = 2
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = 29600 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(out.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    q, db = bf_database(6, 30, 1999)
    whole = [x.tolist() for x in om.bf_top2(q, db)]
    assert res[0] == whole and res[1] == whole


# ---- GPU ----------------------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("kernel", [0, 1], ids=["k_bf_mfma", "k_bf_top2"])
@pytest.mark.parametrize("seed,nq,ndb", [(10, 1000, 100003), (11, 37, 1), (12, 300, 0),
                                         (13, 64, 2), (14, 257, 4099), (15, 1, 65536)])
def test_gpu_bf_top2_parity(orbx_lib, seed, nq, ndb, kernel):
    """Both distance kernels (ORBX_BF_MFMA: +-1 int8 MFMA dot products; ORBX_BF_VALU: XOR +
    v_bcnt, north_star's "no MFMA" form) against the oracle's best / second loop
    (src/ORBmatcher.cc:232-256 over every row; DescriptorDistance :1715-1731)."""
    from my_orb_slam2_amd import ORBmatcher
    q, db = bf_database(seed, nq, ndb)
    m = ORBmatcher(0.75, True)
    m.set_bf_kernel(kernel)
    got = m.hamming_bf_top2(q, db)
    want = om.bf_top2(q, db)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", [0, 1], ids=["k_bf_mfma", "k_bf_top2"])
def test_gpu_bf_top2_device_shards(orbx_lib, gpu, kernel):
    """The device entry point on shards of one database (idx_base = the shard's first row),
    folded by merge_top2 in shard order, equals the whole database's result."""
    from my_orb_slam2_amd import ORBmatcher
    q, db = bf_database(16, 500, 300007)
    m = ORBmatcher(0.75, True)
    m.set_bf_kernel(kernel)
    dq = torch.from_numpy(q).to(gpu)
    ddb = torch.from_numpy(db).to(gpu)
    whole = om.bf_top2(q, db)
    for world in (1, 3, 8):
        parts = []
        for r in range(world):
            r0, r1 = shard_range(len(db), r, world)
            out = [torch.full((len(q),), -7, dtype=torch.int32, device=gpu) for _ in range(3)]
            m.hamming_bf_top2_device(dq, len(q), ddb[r0:], r1 - r0, *out, idx_base=r0)
            parts.append(tuple(out))
        torch.cuda.synchronize(gpu)
        merged = merge_top2(parts)
        for g, w in zip(merged, whole):
            np.testing.assert_array_equal(g.cpu().numpy(), w)
