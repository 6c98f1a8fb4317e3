"""Frame sharding across ranks.

A stream of F frames has F-1 independent pairs (each pair's detect -> match ->
E -> R, t depends only on its two frames; visual_odometry_v3.py:384-408).  The
pairs are split into contiguous per-rank runs; a rank processing pairs
[p0, p1) needs frames [p0, p1] (a one-frame halo on the right, shared with the
next rank, detected twice — the only redundant work).  No data-path
collective: after the batch each rank holds its 256-byte pair records and the
only exchange is one all-gather of those records (RCCL over xGMI on the GPU,
gloo in the CPU tests) to reassemble the pose stream in order.

The absolute pose chain T_abs[p] = T_abs[p-1] . T_rel[p] (v3:367) is a prefix
product; ranks chain their own run from identity and `compose_chain` folds the
per-rank partial products in rank order — equal to the sequential chain up to
floating-point reassociation of the 4x4 products (pinned in tests/test_dist.py).
The marker-scale step also needs the previous pair's projection matrix
(v3:343): with `shard_frames(..., left_halo=True)` a rank also loads frame
p0-1 and computes pair p0-1, whose R|t gives its first pair's P_prev through
the device carry; that extra pair's record is dropped before the gather.
"""
from __future__ import annotations

import numpy as np


def shard_pairs(n_frames: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous pair range [p0, p1) of `rank`; sizes differ by at most one."""
    if n_frames < 2:
        return 0, 0
    pairs = n_frames - 1
    base, extra = divmod(pairs, world)
    p0 = rank * base + min(rank, extra)
    return p0, p0 + base + (1 if rank < extra else 0)


def shard_frames(n_frames: int, world: int, rank: int, left_halo: bool = False) -> tuple[int, int]:
    """Frame range [f0, f1) a rank must load for its pairs (right halo included;
    with left_halo also the frame before its first pair, when there is one)."""
    p0, p1 = shard_pairs(n_frames, world, rank)
    if p1 <= p0:
        return p0, p0
    return (p0 - 1 if left_halo and p0 > 0 else p0), p1 + 1


def max_pairs_per_rank(n_frames: int, world: int) -> int:
    return max(p1 - p0 for p0, p1 in (shard_pairs(n_frames, world, r) for r in range(world)))


def gather_records(records, n_local: int, n_frames: int, group=None):
    """All-gather per-rank pair records (uint8 tensors of n_local x 256 bytes,
    padded to the largest shard) and return them in global pair order as one
    uint8 tensor of (n_frames - 1) x 256 bytes on the records' device."""
    import torch
    import torch.distributed as dist
    from droplet_visual_odometry_amd._native import PAIR_RECORD_DTYPE
    rb = PAIR_RECORD_DTYPE.itemsize
    world = dist.get_world_size(group)
    cap = max_pairs_per_rank(n_frames, world)
    send = torch.zeros(cap * rb, dtype=torch.uint8, device=records.device)
    send[: n_local * rb] = records[: n_local * rb]
    recv = torch.empty(world * cap * rb, dtype=torch.uint8, device=records.device)
    dist.all_gather_into_tensor(recv, send, group=group)
    parts = []
    for r in range(world):
        p0, p1 = shard_pairs(n_frames, world, r)
        parts.append(recv[r * cap * rb: (r * cap + (p1 - p0)) * rb])
    return torch.cat(parts)


def local_chain(T_rel: np.ndarray) -> np.ndarray:
    """Prefix products of [n, 4, 4] relative poses starting from identity."""
    out = np.empty_like(T_rel)
    T = np.eye(4)
    for i in range(len(T_rel)):
        T = T.dot(T_rel[i])
        out[i] = T
    return out


def compose_chain(T0: np.ndarray, shard_chains: list[np.ndarray]) -> np.ndarray:
    """Fold per-rank local chains (each from identity) into the absolute chain
    starting at T0: rank r's poses are left-multiplied by the running product of
    all earlier ranks' last poses."""
    out = []
    acc = np.asarray(T0, np.float64)
    for ch in shard_chains:
        if len(ch) == 0:
            continue
        out.append(np.einsum("ij,njk->nik", acc, ch))
        acc = out[-1][-1]
    return np.concatenate(out) if out else np.zeros((0, 4, 4))
