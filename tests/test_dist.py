"""Frame sharding + record all-gather + pose-chain fold on
world_size 2 with gloo on the CPU (the GPU path swaps gloo for RCCL)."""
import os
import socket

import numpy as np
import pytest

from droplet_visual_odometry_amd import dist as ddist


@pytest.mark.parametrize("n_frames", [0, 1, 2, 3, 8, 129, 1000])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shards_cover_pairs_once(n_frames, world):
    seen = []
    for r in range(world):
        p0, p1 = ddist.shard_pairs(n_frames, world, r)
        f0, f1 = ddist.shard_frames(n_frames, world, r)
        assert p0 <= p1
        if p1 > p0:
            assert (f0, f1) == (p0, p1 + 1) and f1 <= n_frames
            assert ddist.shard_frames(n_frames, world, r, left_halo=True) == (max(0, p0 - 1), p1 + 1)
        seen.extend(range(p0, p1))
    assert seen == list(range(max(0, n_frames - 1)))
    sizes = [np.subtract(*ddist.shard_pairs(n_frames, world, r)[::-1]) for r in range(world)]
    assert max(sizes) - min(sizes) <= 1


def _rand_rigid(rng):
    from droplet_visual_odometry_amd import transformations as tr
    T = tr.euler_matrix(*rng.uniform(-0.2, 0.2, 3))
    T[:3, 3] = rng.uniform(-0.3, 0.3, 3)
    return T


def test_compose_chain_matches_sequential():
    rng = np.random.default_rng(3)
    T_rel = np.stack([_rand_rigid(rng) for _ in range(50)])
    T0 = _rand_rigid(rng)
    seq = ddist.local_chain(T_rel)
    seq = np.einsum("ij,njk->nik", T0, seq)
    ref = []
    T = T0
    for M in T_rel:
        T = T.dot(M)
        ref.append(T)
    np.testing.assert_allclose(seq, np.stack(ref), rtol=0, atol=1e-12)
    for world in (2, 3, 7):
        chains = [ddist.local_chain(T_rel[slice(*ddist.shard_pairs(51, world, r))]) for r in range(world)]
        np.testing.assert_allclose(ddist.compose_chain(T0, chains), np.stack(ref), rtol=0, atol=1e-12)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_frames, out):
    import torch
    import torch.distributed as dist
    from droplet_visual_odometry_amd._native import PAIR_RECORD_DTYPE
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p0, p1 = ddist.shard_pairs(n_frames, world, rank)
    rec = np.zeros(p1 - p0, PAIR_RECORD_DTYPE)
    rec["n_matches"] = np.arange(p0, p1)            # pair id stamped into each record
    rec["t"][:, 0] = np.arange(p0, p1) * 0.5
    rec["status"] = rank
    t = torch.from_numpy(rec.view(np.uint8).copy())
    allrec = ddist.gather_records(t, p1 - p0, n_frames).numpy().view(PAIR_RECORD_DTYPE)
    out[rank] = (allrec["n_matches"].tolist(), allrec["t"][:, 0].tolist(), allrec["status"].tolist())
    dist.destroy_process_group()


@pytest.mark.parametrize("n_frames", [2, 9, 10])
def test_gather_records_gloo_world2(n_frames):
    import torch.multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), n_frames, out), nprocs=2, join=True)
    for r in range(2):
        ids, tx, st = out[r]
        assert ids == list(range(n_frames - 1))
        assert tx == [0.5 * i for i in range(n_frames - 1)]
        want = [0 if i < ddist.shard_pairs(n_frames, 2, 0)[1] else 1 for i in range(n_frames - 1)]
        assert st == want
