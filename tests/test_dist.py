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


@pytest.mark.parametrize("n_pairs,world", [(8, 2), (7, 2), (5, 3)])
def test_shard_window_one_stream(n_pairs, world):
    """Each window pair is computed by exactly one rank; every rank but the one
    holding the stream's first pair loads one halo frame before its run."""
    for first in (0, n_pairs):
        seen = []
        for r in range(world):
            p0, p1, f0, f1, halo = ddist.shard_window(n_pairs, world, r, first)
            seen.extend(range(p0, p1))
            if p1 > p0:
                assert (f0, f1) == (p0 - halo, p1 + 1)
                assert halo == (0 if p0 == 0 else 1)
        assert seen == list(range(first, first + n_pairs))


def _oracle_records(frames, K, n, P0, corners, marker_len):
    """Records + T_rel of consecutive pairs from the oracle (the CPU restatement
    of what FrameStream.process + pose_tail compute), P_prev carried from P0."""
    import oracle
    from droplet_visual_odometry_amd._native import PAIR_RECORD_DTYPE
    pairs = len(frames) - 1
    rec = np.zeros(pairs, PAIR_RECORD_DTYPE)
    T_rel = np.zeros((pairs, 4, 4))
    kp_prev = None
    P, T = P0, np.eye(4)
    for i in range(pairs):
        r = oracle.pair_pose(frames[i], frames[i + 1], K, n, kp_prev=kp_prev)
        kp_prev = (r["kp_cur"], r["desc_cur"])
        rec["R"][i] = r["R"].ravel()
        rec["t"][i] = r["t_unit"].ravel()
        rec["E"][i] = r["E"].ravel()
        rec["n_matches"][i] = len(r["q"])
        rec["ransac_iters"][i] = r["iters"]
        P, T_rel[i], T = oracle.pose_tail(K, r["R"], r["t_unit"], corners[i], corners[i + 1], marker_len, P, T)
    return rec, T_rel


def _sharded_worker(rank, world, port, n_pairs, windows, out):
    import sys
    import torch
    import torch.distributed as dist
    torch.set_num_threads(2)  # two ranks on 8 host cores: oversubscribed torch threads make rendering ~50x slower
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    from conftest import synth_frames
    from droplet_visual_odometry_amd._native import PAIR_RECORD_DTYPE
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = ddist.ShardedPoseStream(world, rank, n_pairs, "cpu")
    rb = PAIR_RECORD_DTYPE.itemsize
    T = np.eye(4)
    got_rec, got_T = [], []
    for w in range(windows):
        p0, p1, f0, f1, halo = ddist.shard_window(n_pairs, world, rank, w * n_pairs)
        frames, K = synth_frames(320, 240, range(f0, f1))
        corners = np.stack([marker_corners(i, K) for i in range(f0, f1)])
        rec, T_rel = _oracle_records(frames, K, 300, K @ np.hstack((np.eye(3), np.zeros((3, 1)))), corners,
                                     MARKER_LEN)
        recs = np.zeros(sh.cap + 1, PAIR_RECORD_DTYPE)
        recs[:len(rec)] = rec
        Ts = np.zeros((sh.cap + 1, 4, 4))
        Ts[:len(T_rel)] = T_rel
        all_rec, all_T = sh.exchange(torch.from_numpy(recs.view(np.uint8).copy()), torch.from_numpy(Ts), halo)
        assert all_rec.numel() == n_pairs * rb and all_T.shape[0] == n_pairs
        for M in all_T.numpy():          # rank 0's chain, sequential as on one rank
            T = T.dot(M)
            got_T.append(T)
        got_rec.append(all_rec.numpy().view(PAIR_RECORD_DTYPE).copy())  # views of the recv buffers
    out[rank] = (np.concatenate(got_rec).tobytes(), np.stack(got_T).tobytes())
    dist.destroy_process_group()


@pytest.mark.parametrize("n_pairs,windows", [(4, 2), (5, 1)])
def test_sharded_one_stream_matches_single_rank_gloo(oracle_mod, n_pairs, windows):
    """One stream sharded over 2 ranks with the left halo: the exchanged records
    (R, t, E, counts) and the chained T_abs equal a single rank's sequential run
    over the same frames, bit for bit (C4, trajectory_evaluation_dual_process.py:172-252)."""
    import torch.multiprocessing as mp
    from conftest import synth_frames
    from droplet_visual_odometry_amd._native import PAIR_RECORD_DTYPE
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_sharded_worker, args=(2, _free_port(), n_pairs, windows, out), nprocs=2, join=True)
    F = n_pairs * windows + 1
    frames, K = synth_frames(320, 240, range(F))
    corners = np.stack([marker_corners(i, K) for i in range(F)])
    rec, T_rel = _oracle_records(frames, K, 300, K @ np.hstack((np.eye(3), np.zeros((3, 1)))), corners, MARKER_LEN)
    T = np.eye(4)
    want_T = []
    for M in T_rel:
        T = T.dot(M)
        want_T.append(T)
    for r in range(2):
        got_rec, got_T = out[r]
        got = np.frombuffer(got_rec, PAIR_RECORD_DTYPE)
        assert got.tobytes() == rec.tobytes()
        np.testing.assert_array_equal(np.frombuffer(got_T).reshape(-1, 4, 4), np.stack(want_T))
