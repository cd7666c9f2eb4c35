"""Multi-GPU plumbing for the sharded matcher workloads.

One process per GPU (torch.distributed; the "nccl" backend is RCCL over xGMI on ROCm, "gloo"
for CPU tests).  The data path never crosses ranks except where the reference's own loop has
an exchange step:

* stereo extract+match (C2): independent frames, no collective (replicas, weak scaling);
* relocalisation (C4): the keyframe database is sharded by keyframe; the query frame's
  descriptors are broadcast from the rank that extracted it and the per-keyframe match counts
  are all-gathered, so every rank sees the candidates with >= 15 matches that
  Tracking::Relocalization keeps (Tracking.cc:1479-1500); the match lists of those
  candidates are then gathered (only they go on to PnP, :1503-1528);
* batched SearchForTriangulation (C5): keyframe-pair jobs are sharded; counts and the per-job
  match arrays are all-gathered;
* brute-force top-2 against a descriptor database (C4, pure BF): the database is sharded by
  row, every rank's top-2 of every query is all-gathered and folded in rank order.
"""
from __future__ import annotations

import numpy as np


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [begin, end) block of n units owned by `rank` (sizes differ by <= 1)."""
    base, extra = divmod(n, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def broadcast_query(tensors, src: int = 0):
    """Send the query frame's arrays (descriptors, angles, ...) from `src` to every rank."""
    import torch.distributed as dist
    for t in tensors:
        dist.broadcast(t, src)
    return tensors


# ---- pure merge functions: what every rank does with the all-gathered shard buffers ----------
# (factored out of the collectives so that a one-device test can run the shards in turn and
# merge them with exactly this code, tests/test_gpu_sharding.py)

def pad_shard(local, n_total: int, world: int):
    """A rank's shard rows in the fixed-size buffer every rank all-gathers (the largest shard
    of shard_range; the tail of a smaller shard is zero)."""
    import torch
    cap = max(e - b for b, e in (shard_range(n_total, r, world) for r in range(world)))
    buf = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    buf[:local.shape[0]] = local
    return buf


def merge_shards(parts, n_total: int, world: int):
    """The per-rank padded buffers (all_gather's output, rank order) as one [n_total, ...]
    tensor in global unit order."""
    import torch
    sizes = [shard_range(n_total, r, world) for r in range(world)]
    return torch.cat([parts[r][:e - b] for r, (b, e) in enumerate(sizes)])


class CandidateOverflow(RuntimeError):
    """A rank found more relocalisation candidates than its block holds; `needed` is the
    largest per-rank count (a block capacity that holds every rank's candidates)."""

    def __init__(self, needed: int, cap: int):
        super().__init__(f"{needed} relocalisation candidates on one rank, block capacity {cap}")
        self.needed = needed
        self.cap = cap


def candidate_block(local_matches, local_counts, k0: int, cap: int = 64, min_matches: int = 15):
    """This rank's relocalisation candidates (keyframes with >= min_matches, Tracking.cc:1487)
    as a fixed [1 + cap, 1 + F] int32 block built on the device without a host round trip.
    Row 0 is a header: (the rank's true candidate count, cap, -1, ...); row 1 + i = (global
    keyframe id, its match list) for the i-th candidate in keyframe order, kf id -1 past the
    last one.  The reference keeps every candidate, so a count above cap is not truncated
    silently: merge_candidate_blocks raises CandidateOverflow from the header, and
    gather_candidate_matches then gathers again with a block that holds them all."""
    import torch
    dev = local_matches.device
    n, F = local_matches.shape
    mask = local_counts[:n] >= min_matches
    order = torch.argsort((~mask).to(torch.int8), stable=True)[:cap]   # candidates first
    k = min(cap, n)
    block = torch.full((1 + cap, 1 + F), -1, dtype=torch.int32, device=dev)
    block[0, 0] = mask.sum().to(torch.int32)
    block[0, 1] = cap
    if k:
        ids = torch.where(mask[order[:k]], order[:k].to(torch.int32) + k0,
                          torch.full((k,), -1, dtype=torch.int32, device=dev))
        block[1:1 + k, 0] = ids
        block[1:1 + k, 1:] = torch.where((ids >= 0)[:, None],
                                         local_matches[order[:k]].to(torch.int32),
                                         torch.full((k, F), -1, dtype=torch.int32, device=dev))
    return block


def merge_candidate_blocks(parts):
    """[(kf_id, matches[F]), ...] in keyframe order from the all-gathered candidate blocks.
    Raises CandidateOverflow if any rank's header counts more candidates than its block
    holds."""
    out = []
    needed, cap = 0, None
    for blk in parts:
        b = blk.cpu().numpy() if hasattr(blk, "cpu") else np.asarray(blk)
        cnt, bcap = int(b[0, 0]), int(b[0, 1])
        if cnt > bcap:
            needed, cap = max(needed, cnt), bcap
        for row in b[1:]:
            if row[0] >= 0:
                out.append((int(row[0]), row[1:]))
    if cap is not None:
        raise CandidateOverflow(needed, cap)
    out.sort(key=lambda t: t[0])
    return out


# ---- collectives ------------------------------------------------------------------------------

def merge_top2(parts):
    """Fold per-shard brute-force top-2 results (best_idx, best_dist, second_dist), given in
    shard order = database row order, into the whole database's: the best is the earlier
    shard's on equal distance (the reference loop's strict `<`, src/ORBmatcher.cc:247), the
    second is the second least distance of the union of the two sorted pairs.  Same
    arithmetic as k_bf_merge (orbx_bf.hip) over its chunks; tensors or numpy arrays."""
    bi, b1, b2 = parts[0]
    lib = np if isinstance(b1, np.ndarray) else __import__("torch")
    for ei, e1, e2 in parts[1:]:
        b2 = lib.minimum(lib.maximum(b1, e1), lib.minimum(b2, e2))
        take = e1 < b1
        bi = lib.where(take, ei, bi)
        b1 = lib.where(take, e1, b1)
    return bi, b1, b2


def gather_top2(best_idx, best_dist, second_dist, world: int):
    """All-gather every rank's top-2 over its database shard (global row numbers, see
    orbx_hamming_bf_top2_device's idx_base) and fold them in rank order: 12 bytes per query
    and rank cross the links (pure BF)."""
    import torch
    import torch.distributed as dist
    loc = torch.stack([best_idx, best_dist, second_dist])
    parts = [torch.empty_like(loc) for _ in range(world)]
    dist.all_gather(parts, loc)
    return merge_top2([(p[0], p[1], p[2]) for p in parts])


def all_gather_counts(local, n_total: int, world: int):
    """All-gather per-unit counts of every rank's shard into one [n_total] tensor in global
    unit order (shards are the contiguous blocks of shard_range)."""
    import torch
    import torch.distributed as dist
    buf = pad_shard(local, n_total, world)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    return merge_shards(parts, n_total, world)


def relocalisation_candidates(counts, min_matches: int = 15) -> np.ndarray:
    """Keyframes whose SearchByBoW found at least 15 matches (Tracking.cc:1487-1491)."""
    c = counts.cpu().numpy() if hasattr(counts, "cpu") else np.asarray(counts)
    return np.nonzero(c >= min_matches)[0]


def gather_rows(local, n_total: int, world: int):
    """All-gather the rows of every rank's shard (a [n_local, ...] tensor; shards are the
    contiguous blocks of shard_range) into one [n_total, ...] tensor in global order."""
    import torch
    import torch.distributed as dist
    buf = pad_shard(local, n_total, world)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    return merge_shards(parts, n_total, world)


def gather_candidate_blocks(local_matches, local_counts, k0: int, world: int, cap: int = 64,
                            min_matches: int = 15):
    """All-gather every rank's candidate block (candidate_block): world [1 + cap, 1 + F] device
    tensors, built and exchanged with no host synchronisation (so it can sit inside a timed
    step); merge_candidate_blocks decodes it afterwards."""
    import torch
    import torch.distributed as dist
    blk = candidate_block(local_matches, local_counts, k0, cap, min_matches)
    parts = [torch.empty_like(blk) for _ in range(world)]
    dist.all_gather(parts, blk)
    return parts


def gather_candidate_matches(local_matches, counts, n_total: int, world: int,
                             min_matches: int = 15, cap: int = 64):
    """The match lists of the relocalisation candidates collected from the ranks that own
    them: [(kf_id, matches[F]), ...] in keyframe order on every rank.  `counts` is this
    rank's shard counts or the all-gathered [n_total] counts.  Every rank reads the same
    gathered headers, so on an overflow all ranks gather again together, with a block sized to
    the largest rank's count: no candidate is dropped (Tracking.cc:1479-1500 keeps them all)."""
    import torch.distributed as dist
    rank = dist.get_rank()
    b, e = shard_range(n_total, rank, world)
    local_counts = counts[b:e] if counts.shape[0] == n_total else counts
    parts = gather_candidate_blocks(local_matches, local_counts, b, world, cap, min_matches)
    try:
        return merge_candidate_blocks(parts)
    except CandidateOverflow as ov:
        parts = gather_candidate_blocks(local_matches, local_counts, b, world, ov.needed,
                                        min_matches)
        return merge_candidate_blocks(parts)
