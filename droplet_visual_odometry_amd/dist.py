"""Frame sharding across ranks.

A stream of F frames has F-1 independent pairs (each pair's detect -> match ->
E -> R, t depends only on its two frames; visual_odometry_v3.py:384-408).  The
pairs are split into contiguous per-rank runs; a rank processing pairs
[p0, p1) needs frames [p0, p1] (a one-frame halo on the right, shared with the
next rank, detected twice — the only redundant work).  No data-path
collective: after the batch each rank holds its 256-byte pair records.

Two things couple adjacent pairs, both cheap and both downstream of the
records: the marker-scale step of pair p triangulates against the previous
*successful* pair's projection P = K [R | t] (v3:264-265, :344), and the
absolute pose is the prefix product T_abs[p] = T_abs[p-1] . T_rel[p] (v3:367).
So the exchange is one all-gather of each rank's records plus the marker
corners of its pairs (`ShardedPoseStream`), and rank 0 runs the whole pose
tail over the window in pair order from the gathered records
(`stream.PoseTail` -> dvo_pose_tail_records: the same kernels and the same
record fields as the single-rank dvo_stream_pose_tail).  P_prev of a rank's
first pair is then the last successful pair's wherever it was computed —
including when the pairs at a shard boundary fail — so records, T_rel and
T_abs are bit-identical to one rank processing the whole stream.

The host helpers `local_chain` / `compose_chain` fold per-rank partial
products instead (equal up to reassociation, tests/test_dist.py).
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


def shard_frames(n_frames: int, world: int, rank: int) -> tuple[int, int]:
    """Frame range [f0, f1) a rank must load for its pairs (right halo included)."""
    p0, p1 = shard_pairs(n_frames, world, rank)
    if p1 <= p0:
        return p0, p0
    return p0, p1 + 1


def max_pairs_per_rank(n_frames: int, world: int) -> int:
    return max(p1 - p0 for p0, p1 in (shard_pairs(n_frames, world, r) for r in range(world)))


def shard_window(n_pairs: int, world: int, rank: int, first_pair: int = 0):
    """`rank`'s share of a window of `n_pairs` consecutive pairs of ONE stream
    starting at global pair `first_pair`: (p0, p1, f0, f1) -- pairs [p0, p1)
    and the frames [f0, f1) = [p0, p1 + 1) to load (pair p is frames p, p+1)."""
    a, b = shard_pairs(n_pairs + 1, world, rank)
    p0, p1 = first_pair + a, first_pair + b
    if p1 <= p0:
        return p0, p0, p0, p0
    return p0, p1, p0, p1 + 1


class ShardedPoseStream:
    """The exchange step of one pose stream sharded across ranks (SURVEY.md
    §8e, BASELINE configs[3]): windows of `window_pairs` pairs, each rank
    computing its `shard_window` run on its own GPU.

    One send buffer per instance holds the rank's records (`records`, where
    FrameStream.process writes them: capacity `cap` pairs) followed by its
    pairs' marker corners (`set_corners`: previous-frame and current-frame
    corners, k x 2 doubles each, as the harness passes them to
    visual_odometry_calculations, trajectory_evaluation_dual_process.py:158-164).
    `exchange()` all-gathers the send buffers in one collective (RCCL over
    xGMI; gloo through host memory with host_gather=True) and returns the
    window's records, previous and current corners in global pair order as
    new contiguous tensors on `device`.

    Ordering contract (RCCL): the collective runs on torch's current stream.
    Before it, that stream must wait for the library stream that wrote
    `records`; before the next write into `records`, the library stream must
    wait for `exchange`'s `done` event (bench.py main_sharded)."""

    def __init__(self, world: int, rank: int, window_pairs: int, device, k: int = 4, group=None,
                 host_gather: bool = False):
        import torch
        from droplet_visual_odometry_amd._native import PAIR_RECORD_DTYPE
        self.world, self.rank, self.window_pairs, self.group, self.k = world, rank, window_pairs, group, k
        self.device = torch.device(device)
        self.rb = PAIR_RECORD_DTYPE.itemsize
        self.cb = k * 2 * 8                       # one frame's corners
        self.counts = [b - a for a, b in (shard_pairs(window_pairs + 1, world, r) for r in range(world))]
        self.cap = max(self.counts)
        self.n_local = self.counts[rank]
        self.seg = self.cap * (self.rb + 2 * self.cb)
        self.host_gather = host_gather
        self.send = torch.zeros(self.seg, dtype=torch.uint8, device=self.device)
        gdev = torch.device("cpu") if host_gather else self.device
        self.recv = torch.empty(world * self.seg, dtype=torch.uint8, device=gdev)
        self.done = None  # torch.cuda.Event recorded after the last collective (device gathers)
        # the second exchange: T_rel of each rank's own pairs (dvo_pose_rel_range), gathered for rank 0's chain
        self.p0_local = sum(self.counts[:rank])
        self.T_send = torch.zeros((self.cap, 4, 4), dtype=torch.float64, device=self.device)
        # rank 0 gathers the shards (exchange_T); the others only send
        self.T_recv = torch.empty((world if rank == 0 else 1, self.cap, 4, 4), dtype=torch.float64, device=gdev)

    @property
    def records(self):
        """The rank's record slots (uint8, cap x 256 B) inside the send buffer."""
        return self.send[:self.cap * self.rb]

    def _corner_block(self, which: int):
        o = self.cap * self.rb + which * self.cap * self.cb
        return self.send[o:o + self.cap * self.cb].view(__import__("torch").float64).view(self.cap, self.k, 2)

    def set_corners(self, c_prev, c_cur):
        """Copy the rank's per-pair corners ([n_local, k, 2] float64) into the
        send buffer (on torch's current stream)."""
        n = self.n_local
        if tuple(c_prev.shape) != (n, self.k, 2) or tuple(c_cur.shape) != (n, self.k, 2):
            raise ValueError(f"corners must be [{n}, {self.k}, 2]")
        self._corner_block(0)[:n].copy_(c_prev, non_blocking=True)
        self._corner_block(1)[:n].copy_(c_cur, non_blocking=True)

    def exchange(self):
        import torch
        import torch.distributed as dist
        send = self.send.cpu() if self.host_gather else self.send
        dist.all_gather_into_tensor(self.recv, send, group=self.group)
        if not self.host_gather and self.recv.is_cuda:
            self.done = torch.cuda.Event()
            self.done.record(torch.cuda.current_stream(self.recv.device))
        v = self.recv.view(self.world, self.seg)
        rb, cb, cap = self.rb, self.cb, self.cap
        recs = torch.cat([v[r, :c * rb] for r, c in enumerate(self.counts)])
        cp = torch.cat([v[r, cap * rb:cap * rb + c * cb] for r, c in enumerate(self.counts)])
        cc = torch.cat([v[r, cap * (rb + cb):cap * (rb + cb) + c * cb] for r, c in enumerate(self.counts)])
        n = self.window_pairs
        cp = cp.view(torch.float64).view(n, self.k, 2)
        cc = cc.view(torch.float64).view(n, self.k, 2)
        if self.host_gather:
            recs, cp, cc = (x.to(self.device) for x in (recs, cp, cc))
        return recs, cp, cc

    def exchange_T(self):
        """Gather every rank's T_rel (T_send[:n_local]) to rank 0, the only rank that chains, and
        return the window's T_rel in pair order there ([window_pairs, 4, 4] on `device`); None on
        the other ranks.  One gather: rank 0 receives (world - 1) shards and no other rank
        receives anything (an all-gather would send every shard to every rank)."""
        import torch
        import torch.distributed as dist
        send = self.T_send.cpu() if self.host_gather else self.T_send
        if self.world == 1:
            self.T_recv[0].copy_(send)
        else:
            dist.gather(send, list(self.T_recv.unbind(0)) if self.rank == 0 else None, dst=0, group=self.group)
        if self.rank != 0:
            return None
        T = torch.cat([self.T_recv[r, :c] for r, c in enumerate(self.counts)])
        return T.to(self.device) if self.host_gather else T


class ShardedStreamRunner:
    """One rank's loop over a sharded pose stream (bench.py main_sharded and
    tests/test_gpu_sharded.py run this same code): `streams` library streams,
    window w on stream w mod streams, each window's batch submitted pipelined
    (FrameStream.submit: its RANSAC rounds run merged with the stream's next
    pipeline_depth() - 1 windows'), so a window's records are complete -- and
    exchanged -- when it retires.  Every (stream, in-flight slot) has its own
    ShardedPoseStream send buffer; the library writes the window's records
    straight into it.  Rank 0 keeps one PoseTail whose carry continues across
    windows.

    `step(frames, c_prev, c_cur)` submits one window: frames = the rank's
    n_local + 1 device frames, c_prev / c_cur its n_local pairs' corners.
    Returns the windows retired by this step, oldest first (one per step once
    prime_steps windows are in flight), each as (records, T_rel, T_abs): the
    window's gathered records (every rank) and rank 0's relative poses (device)
    and absolute poses (a concurrent.futures.Future of the host [n, 4, 4]
    array, chained on a host thread; None elsewhere), valid until the window's
    send slot retires again (streams x pipeline_depth() steps later).
    `drain()` retires the windows still in flight the same way.  Every rank
    calls step / drain in the same order, so the collectives line up.

    The pose tail is split: every rank computes the relative poses of its own
    pairs from the gathered records (dvo_pose_rel_range: the marker scale
    triangulates against the last successful pair before it, wherever that
    was computed), a second all-gather brings the window's T_rel to rank 0,
    and rank 0 runs only the serial absolute chain, on a host thread
    (dvo_pose_chain_host: one sequential product per pair, ~50 ns on a CPU
    core while the GPU runs the next batches); the poses equal one rank's
    pose tail over the stream bit for bit.

    Ordering without host syncs on the device-gather path: the library stream
    waits for the slot's previous collective before writing its records;
    torch's stream waits for the records before the collective; the tail
    halves and the second collective follow on torch's stream
    (ordered_side_stream)."""

    def __init__(self, width: int, height: int, K, nfeatures: int, window_pairs: int, world: int, rank: int,
                 marker_length: float, ctx=None, device=None, max_iters: int = 1000, streams: int = 2, k: int = 4,
                 host_gather: bool = False, group=None):
        import collections
        import torch
        from droplet_visual_odometry_amd._native import Context
        from droplet_visual_odometry_amd.stream import FrameStream, HostPoseChain, PoseTail
        self.ctx = ctx if ctx is not None else Context(0 if device is None else device)
        dev = torch.device("cuda", self.ctx.device)
        self.S, self.rank, self.host_gather = max(1, streams), rank, host_gather
        self.D = FrameStream.pipeline_depth()
        self.shs = [[ShardedPoseStream(world, rank, window_pairs, dev, k=k, group=group, host_gather=host_gather)
                     for _ in range(self.D)] for _ in range(self.S)]
        self.n_local = self.shs[0][0].n_local
        self.fss = [FrameStream(width, height, K, nfeatures=nfeatures, max_frames=self.n_local + 1,
                                max_iters=max_iters, ctx=self.ctx) for _ in range(self.S)]
        # every rank: the P_prev carry and its own pairs' T_rel; rank 0 also the chain, on the host
        self.tail = PoseTail(K, marker_length, ctx=self.ctx)
        self.chain = HostPoseChain(window_pairs, self.S * self.D + 1, dev) if rank == 0 else None
        self.fifo = [collections.deque() for _ in range(self.S)]  # (send slot, global window number) in flight
        self.nsub = [0] * self.S
        self.i = 0
        self.prime_steps = self.S * (self.D - 1)

    def reset_pose(self, P0=None, T0=None):
        """Carry-in of the whole pose stream: P_prev (3x4, default K[I|0]) on every rank's tail and
        the absolute pose T0 (4x4, default identity) of rank 0's chain, before the next window."""
        self.tail.reset(P0, None)
        if self.chain is not None:
            self.chain.reset(T0)

    def step(self, frames, c_prev, c_cur, wait_torch: bool = True):
        """wait_torch (default): order the library stream after work queued on
        torch's current stream -- the frames' producer and, on a slot's first
        use, the zero-fill of its send buffer.  Pass False only for frames that
        are already resident (a slot's first use is still ordered)."""
        k = self.i % self.S
        fs = self.fss[k]
        sh = self.shs[k][self.nsub[k] % self.D]
        first_use = self.nsub[k] < self.D
        self.nsub[k] += 1
        if frames.shape[0] != self.n_local + 1:
            raise ValueError(f"rank {self.rank} needs {self.n_local + 1} frames per window")
        fs.wait_event(sh.done)  # the slot's previous collective has read its send buffer
        sh.set_corners(c_prev, c_cur)  # torch's stream, after that collective
        self.fifo[k].append((sh, self.i))
        self.i += 1
        retired = fs.submit(frames, sh.records, wait_torch=wait_torch or first_use)
        return [self._exchange(k, self.fifo[k].popleft()[0]) for _ in retired]

    def drain(self):
        done = []
        for k, fs in enumerate(self.fss):
            for _ in fs.drain():
                sh, g = self.fifo[k].popleft()
                done.append((g, k, sh))
        return [self._exchange(k, sh) for _, k, sh in sorted(done, key=lambda t: t[0])]

    def _exchange(self, k, sh):
        import torch
        fs = self.fss[k]
        if self.host_gather:
            fs.sync()
        else:
            torch.cuda.current_stream(fs.device).wait_event(fs.record_event())
        recs, cp, cc = sh.exchange()
        # the pair-parallel half of the tail on every rank, over its own pairs of the window
        self.tail.rel_range(recs, cp, cc, sh.p0_local, sh.n_local, sh.T_send)
        T_rel = sh.exchange_T()
        if self.rank != 0:
            return recs, None, None
        # the serial chain on a host thread (dvo_pose_chain_host): off the GPU, which goes on with the
        # next windows; T_abs is a Future of the host array
        return recs, T_rel, self.chain.submit(T_rel)

    def sync(self):
        import torch
        for f in self.fss:
            f.sync()
        torch.cuda.synchronize()
        if self.chain is not None:
            self.chain.wait()

    def close(self):
        for f in self.fss:
            f.close()
        if self.chain is not None:
            self.chain.close()


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
