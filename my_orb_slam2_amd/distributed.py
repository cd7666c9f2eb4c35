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
  match arrays are all-gathered.
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


def all_gather_counts(local, n_total: int, world: int):
    """All-gather per-unit counts of every rank's shard into one [n_total] tensor in global
    unit order (shards are the contiguous blocks of shard_range)."""
    import torch
    import torch.distributed as dist
    sizes = [shard_range(n_total, r, world) for r in range(world)]
    cap = max(e - b for b, e in sizes)
    buf = torch.zeros(cap, dtype=local.dtype, device=local.device)
    buf[:local.numel()] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    return torch.cat([parts[r][:e - b] for r, (b, e) in enumerate(sizes)])


def relocalisation_candidates(counts, min_matches: int = 15) -> np.ndarray:
    """Keyframes whose SearchByBoW found at least 15 matches (Tracking.cc:1487-1491)."""
    c = counts.cpu().numpy() if hasattr(counts, "cpu") else np.asarray(counts)
    return np.nonzero(c >= min_matches)[0]


def gather_rows(local, n_total: int, world: int):
    """All-gather the rows of every rank's shard (a [n_local, ...] tensor; shards are the
    contiguous blocks of shard_range) into one [n_total, ...] tensor in global order."""
    import torch
    import torch.distributed as dist
    sizes = [shard_range(n_total, r, world) for r in range(world)]
    cap = max(e - b for b, e in sizes)
    buf = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    buf[:local.shape[0]] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    return torch.cat([parts[r][:e - b] for r, (b, e) in enumerate(sizes)])


def gather_candidate_matches(local_matches, counts, n_total: int, world: int,
                             min_matches: int = 15):
    """The match lists of the relocalisation candidates (keyframes with >= min_matches, from
    the all-gathered counts) collected from the ranks that own them.  local_matches is this
    rank's [n_local, F] SearchByBoW output (keyframe-local feature index per frame feature, or
    -1).  Every rank receives [(kf_id, matches[F]), ...] in keyframe order; only the
    candidates travel (a [cap, 1 + F] int32 block per rank, cap = the largest per-rank
    candidate count)."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank()
    c = counts.cpu().numpy() if hasattr(counts, "cpu") else np.asarray(counts)
    sizes = [shard_range(n_total, r, world) for r in range(world)]
    per_rank = [np.nonzero(c[b:e] >= min_matches)[0] + b for b, e in sizes]
    cap = max(1, max(len(p) for p in per_rank))
    F = local_matches.shape[1]
    buf = torch.full((cap, 1 + F), -1, dtype=torch.int32, device=local_matches.device)
    mine = per_rank[rank]
    if len(mine):
        b0 = sizes[rank][0]
        idx = torch.as_tensor(mine - b0, dtype=torch.long, device=local_matches.device)
        buf[:len(mine), 0] = torch.as_tensor(mine, dtype=torch.int32, device=buf.device)
        buf[:len(mine), 1:] = local_matches.index_select(0, idx).to(torch.int32)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    out = []
    for r in range(world):
        for i in range(len(per_rank[r])):
            row = parts[r][i]
            out.append((int(row[0].item()), row[1:]))
    return out
