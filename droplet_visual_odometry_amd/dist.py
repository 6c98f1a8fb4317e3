"""Frame sharding across ranks.

A stream of F frames has F-1 independent pairs (each pair's detect -> match ->
E -> R, t depends only on its two frames; visual_odometry_v3.py:384-408).  The
pairs are split into contiguous per-rank runs; a rank processing pairs
[p0, p1) needs frames [p0, p1] (a one-frame halo on the right, shared with the
next rank, detected twice — the only redundant work).  No data-path
collective: after the batch each rank holds its 256-byte pair records and the
only exchange is one all-gather of those records (RCCL over xGMI on the GPU,
gloo in the CPU tests) to reassemble the pose stream in order.

The marker-scale step of pair p needs the previous pair's projection matrix
P = K [R | t] (v3:264-265, :344).  So a rank whose run starts at p0 > 0 also
loads frame p0-1 (the left halo, `shard_window`) and computes pair p0-1: its
R|t is P_prev for p0, exactly as on one rank, and its record and T_rel are
dropped before the exchange.  (On one rank P_prev is the last *successful*
pair's; the halo reproduces that whenever the halo pair itself succeeds, i.e.
unless frame p0-1 or p0 has no features.)

`ShardedPoseStream.exchange` all-gathers every rank's records and T_rel rows in
pair order; rank 0 then chains T_abs[p] = T_abs[p-1] . T_rel[p] (v3:367) over
the whole window on the device (`stream.PoseChain`, the same left-to-right
4x4 arithmetic as the single-rank pose tail, so T_abs is bit-identical).  The
host helpers `local_chain` / `compose_chain` fold per-rank partial products
instead (equal up to reassociation, tests/test_dist.py).
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


def shard_window(n_pairs: int, world: int, rank: int, first_pair: int = 0):
    """`rank`'s share of a window of `n_pairs` consecutive pairs of ONE stream
    starting at global pair `first_pair`: (p0, p1, f0, f1, halo) -- pairs
    [p0, p1), frames [f0, f1) to load (pair p is frames p, p+1) and halo = 1
    when frame p0-1 is loaded too, so that the rank's first computed pair is
    the dropped halo pair p0-1."""
    a, b = shard_pairs(n_pairs + 1, world, rank)
    p0, p1 = first_pair + a, first_pair + b
    if p1 <= p0:
        return p0, p0, p0, p0, 0
    halo = 1 if p0 > 0 else 0
    return p0, p1, p0 - halo, p1 + 1, halo


class ShardedPoseStream:
    """The exchange step of one pose stream sharded across ranks (SURVEY.md
    §8e, BASELINE configs[3]): windows of `window_pairs` pairs, each rank
    computing its `shard_window` run (halo pair first) on its own GPU.

    `exchange(records, T_rel, halo)` takes the rank's computed records
    (uint8, 256 B per pair, halo pair first) and T_rel ([pairs, 4, 4] float64)
    and returns the window's records and T_rel in global pair order on every
    rank: one all-gather each (RCCL over xGMI; gloo through host memory with
    host_gather=True).  Inputs are sliced in place, so the gathered sends are
    the rank's buffers themselves: they must hold at least halo + cap pairs,
    cap = max pairs per rank.  The returned tensors are views of the receive
    buffers (no copy when the shards are equal), valid until the next exchange."""

    def __init__(self, world: int, rank: int, window_pairs: int, device, group=None, host_gather: bool = False):
        import torch
        from droplet_visual_odometry_amd._native import PAIR_RECORD_DTYPE
        self.world, self.rank, self.window_pairs, self.group = world, rank, window_pairs, group
        self.rb = PAIR_RECORD_DTYPE.itemsize
        self.counts = [b - a for a, b in (shard_pairs(window_pairs + 1, world, r) for r in range(world))]
        self.cap = max(self.counts)
        self.n_local = self.counts[rank]
        self.host_gather = host_gather
        gdev = torch.device("cpu") if host_gather else torch.device(device)
        self.recv_rec = torch.empty(world * self.cap * self.rb, dtype=torch.uint8, device=gdev)
        self.recv_T = torch.empty((world * self.cap, 4, 4), dtype=torch.float64, device=gdev)

    def exchange(self, records, T_rel, halo: int):
        import torch.distributed as dist
        rb, cap = self.rb, self.cap
        if records.numel() < (halo + cap) * rb or T_rel.shape[0] < halo + cap:
            raise ValueError(f"buffers must hold halo + {cap} pairs")
        send_rec = records[halo * rb:(halo + cap) * rb]
        send_T = T_rel[halo:halo + cap]
        if self.host_gather:
            send_rec, send_T = send_rec.cpu(), send_T.cpu()
        dist.all_gather_into_tensor(self.recv_rec, send_rec, group=self.group)
        dist.all_gather_into_tensor(self.recv_T.view(-1), send_T.reshape(-1), group=self.group)
        if all(c == cap for c in self.counts):
            return self.recv_rec, self.recv_T
        import torch
        recs = torch.cat([self.recv_rec[r * cap * rb:(r * cap + c) * rb] for r, c in enumerate(self.counts)])
        Ts = torch.cat([self.recv_T[r * cap:r * cap + c] for r, c in enumerate(self.counts)])
        return recs, Ts


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
