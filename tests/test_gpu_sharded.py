"""One stream sharded across ranks on the GPU (BASELINE configs[3], SURVEY.md
§8e): each rank runs FrameStream.process + pose_tail on its run of pairs with
the left halo frame, the ranks exchange records and T_rel
(dist.ShardedPoseStream; gloo through host memory here, since the two ranks
share the box's one GPU — RCCL in bench.py on a multi-GPU node), and rank 0
chains T_abs on the device (stream.PoseChain).  The result must equal one rank
processing the whole stream: records, T_rel and T_abs bit for bit
(trajectory_evaluation_dual_process.py:172-252 is the single-stream loop;
visual_odometry_v3.py:264, :344, :367 couple adjacent pairs)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, NF = 640, 480, 500


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_pairs, windows, out):
    import faulthandler
    import sys
    import torch
    faulthandler.enable()
    import torch.distributed as dist
    torch.set_num_threads(2)
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    from conftest import synth_frames
    from droplet_visual_odometry_amd import dist as ddist
    from droplet_visual_odometry_amd._native import Context
    from droplet_visual_odometry_amd.stream import FrameStream, PoseChain
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    F = n_pairs * windows + 1
    frames, K = synth_frames(W, H, range(F))
    dev = torch.device("cuda", 0)
    d_frames = torch.from_numpy(frames).to(dev)
    d_corners = torch.from_numpy(np.stack([marker_corners(i, K) for i in range(F)])).to(dev)
    ctx = Context(0)
    sh = ddist.ShardedPoseStream(world, rank, n_pairs, dev, host_gather=True)
    fs = FrameStream(W, H, K, nfeatures=NF, max_frames=sh.cap + 2, ctx=ctx)
    fs.reset_pose()
    recs = fs.new_records(sh.cap + 1)
    T_rel = torch.zeros((sh.cap + 1, 4, 4), dtype=torch.float64, device=dev)
    T_abs = torch.zeros((sh.cap + 1, 4, 4), dtype=torch.float64, device=dev)
    chain = PoseChain(ctx)
    got_rec, got_Trel, got_Tabs = [], [], []
    for w in range(windows):
        p0, p1, f0, f1, halo = ddist.shard_window(n_pairs, world, rank, w * n_pairs)
        fs.process(d_frames[f0:f1], recs)
        fs.pose_tail(d_corners[f0:f1 - 1], d_corners[f0 + 1:f1], MARKER_LEN, T_rel, T_abs)
        fs.sync()
        all_rec, all_T = sh.exchange(recs, T_rel, halo)
        got_rec.append(all_rec.numpy().copy())
        got_Trel.append(all_T.numpy().copy())
        if rank == 0:
            got_Tabs.append(chain.run(all_T.to(dev).contiguous()).cpu().numpy())
    torch.cuda.synchronize()
    out[rank] = (np.concatenate(got_rec).tobytes(), np.concatenate(got_Trel).tobytes(),
                 np.concatenate(got_Tabs).tobytes() if got_Tabs else b"")
    fs.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_pairs,windows", [(6, 2), (5, 1)])
def test_sharded_stream_equals_single_rank(gpu_ctx, n_pairs, windows):
    import torch
    import torch.multiprocessing as mp
    from conftest import synth_frames
    from droplet_visual_odometry_amd.stream import FrameStream
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    F = n_pairs * windows + 1
    frames, K = synth_frames(W, H, range(F))
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), n_pairs, windows, out), nprocs=2, join=True)
    fs = FrameStream(W, H, K, nfeatures=NF, max_frames=F, ctx=gpu_ctx)
    fs.reset_pose()
    rec = fs.process(torch.from_numpy(frames).cuda())
    dc = torch.from_numpy(np.stack([marker_corners(i, K) for i in range(F)])).cuda()
    T_rel, T_abs = fs.pose_tail(dc[:-1], dc[1:], MARKER_LEN)
    fs.sync()
    want_rec = rec.cpu().numpy().tobytes()
    want_Trel = T_rel.cpu().numpy()
    want_Tabs = T_abs.cpu().numpy()
    fs.close()
    for r in range(2):
        got_rec, got_Trel, got_Tabs = out[r]
        assert got_rec == want_rec, f"rank {r}: gathered records differ from the single-rank stream"
        np.testing.assert_array_equal(np.frombuffer(got_Trel).reshape(-1, 4, 4), want_Trel)
    got_Tabs = np.frombuffer(out[0][2]).reshape(-1, 4, 4)
    bad = [i for i in range(len(want_Tabs)) if not np.array_equal(got_Tabs[i], want_Tabs[i])]
    assert not bad, f"rank 0 chained T_abs differs at pairs {bad}"


def test_pose_chain_equals_pose_tail_chain(gpu_ctx):
    """dvo_pose_chain over the pose tail's own T_rel, in two pieces with the
    carry in between, gives the pose tail's T_abs bit for bit."""
    import torch
    from conftest import synth_frames
    from droplet_visual_odometry_amd.stream import FrameStream, PoseChain
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    frames, K = synth_frames(W, H, range(6))
    fs = FrameStream(W, H, K, nfeatures=NF, max_frames=6, ctx=gpu_ctx)
    fs.reset_pose()
    fs.process(torch.from_numpy(frames).cuda())
    dc = torch.from_numpy(np.stack([marker_corners(i, K) for i in range(6)])).cuda()
    T_rel, T_abs = fs.pose_tail(dc[:-1], dc[1:], MARKER_LEN)
    fs.sync()
    ch = PoseChain(gpu_ctx)
    a = ch.run(T_rel[:2].contiguous())
    b = ch.run(T_rel[2:].contiguous())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(torch.cat([a, b]).cpu().numpy(), T_abs.cpu().numpy())
    np.testing.assert_array_equal(ch.carry.cpu().numpy().reshape(4, 4), T_abs[-1].cpu().numpy())
    fs.close()


def test_pose_tail_skips_failed_pairs(gpu_ctx, oracle_mod):
    """A pair that fails (no features: the reference raises before
    previous_projection_matrix is set, v3:344) leaves P_prev and T_abs as they
    were; the next good pair triangulates against the last good pair's P."""
    import torch
    from conftest import synth_frames
    from droplet_visual_odometry_amd.stream import FrameStream
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    frames, K = synth_frames(W, H, range(4))
    blank = np.full((H, W), 90, np.uint8)
    seq = np.stack([frames[0], frames[1], blank, frames[2], frames[3]])
    cidx = [0, 1, 1, 2, 3]  # the blank frame keeps frame 1's corners
    corners = np.stack([marker_corners(i, K) for i in cidx])
    fs = FrameStream(W, H, K, nfeatures=NF, max_frames=5, ctx=gpu_ctx)
    fs.reset_pose()
    rec = fs.process(torch.from_numpy(seq).cuda())
    dc = torch.from_numpy(corners).cuda()
    T_rel, T_abs = fs.pose_tail(dc[:-1], dc[1:], MARKER_LEN)
    fs.sync()
    recs = FrameStream.records_numpy(rec, 4)
    assert [int(s) for s in recs["status"]] == [0, -2, -2, 0]
    T_rel, T_abs = T_rel.cpu().numpy(), T_abs.cpu().numpy()
    P, T = K @ np.hstack((np.eye(3), np.zeros((3, 1)))), np.eye(4)
    for p in range(4):
        if recs["status"][p] != 0:
            np.testing.assert_array_equal(T_rel[p], np.eye(4))
            np.testing.assert_allclose(T_abs[p], T, rtol=1e-9, atol=1e-12)
            continue
        P, Tr, T = oracle_mod.pose_tail(K, recs["R"][p].reshape(3, 3), recs["t"][p], corners[p], corners[p + 1],
                                        MARKER_LEN, P, T)
        np.testing.assert_allclose(T_rel[p], Tr, rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(T_abs[p], T, rtol=1e-9, atol=1e-12)
    fs.close()
