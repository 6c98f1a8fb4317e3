"""One stream sharded across ranks on the GPU (BASELINE configs[3], SURVEY.md
§8e): each rank runs FrameStream.process on its run of pairs, the ranks
all-gather records and marker corners (dist.ShardedPoseStream; gloo through
host memory here, since two ranks share the box's one GPU; RCCL at world size
1 below, and across GPUs in bench.py on a multi-GPU node), and rank 0 runs the
window's pose tail from the gathered records (stream.PoseTail).  The result
must equal one rank processing the whole stream: records, T_rel and T_abs bit
for bit (trajectory_evaluation_dual_process.py:172-252 is the single-stream
loop; visual_odometry_v3.py:264, :344, :367 couple adjacent pairs) -- also
when featureless frames make the pairs at a shard boundary fail."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, NF = 640, 480, 500  # the single-rank pose-tail tests below


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stream(W, H, F, blank):
    """F synthetic frames + marker corners; frames in `blank` are featureless
    and keep the previous frame's corners."""
    from conftest import synth_frames
    from droplet_visual_odometry_amd.synth import marker_corners
    frames, K = synth_frames(W, H, range(F))
    frames = frames.copy()
    corners = [marker_corners(i, K) for i in range(F)]
    for b in blank:
        frames[b] = 90
        corners[b] = corners[b - 1]
    return frames, np.stack(corners), K


def _worker(rank, world, port, backend, W, H, NF, n_pairs, windows, blank, streams, out, T0=None):
    import faulthandler
    import sys
    import torch
    faulthandler.enable()
    import torch.distributed as dist
    torch.set_num_threads(2)
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    from droplet_visual_odometry_amd import dist as ddist
    from droplet_visual_odometry_amd._native import Context
    from droplet_visual_odometry_amd.synth import MARKER_LEN
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    frames, corners, K = _stream(W, H, n_pairs * windows + 1, blank)
    d_frames = torch.from_numpy(frames).to(dev)
    d_corners = torch.from_numpy(corners).to(dev)
    run = ddist.ShardedStreamRunner(W, H, K, NF, n_pairs, world, rank, MARKER_LEN, ctx=Context(0),
                                    streams=streams, host_gather=backend == "gloo")
    if T0 is not None:
        run.reset_pose(None, T0)
    got_rec, got_Trel, got_Tabs = [], [], []
    pending = []

    def keep(outs):
        # device copies on torch's stream (ordered after the collective / the tail), read back
        # only at the end: no host sync between windows, so slots are reused while in flight
        for recs, T_rel, T_abs in outs:  # T_abs: rank 0's Future of the host-chained poses
            pending.append((recs.clone(), T_rel.clone() if T_rel is not None else None, T_abs))

    for w in range(windows):
        p0, p1, f0, f1 = ddist.shard_window(n_pairs, world, rank, w * n_pairs)
        keep(run.step(d_frames[f0:f1], d_corners[f0:f1 - 1], d_corners[f0 + 1:f1]))
    keep(run.drain())
    run.sync()
    for recs, T_rel, T_abs in pending:
        got_rec.append(recs.cpu().numpy())
        if T_rel is not None:
            got_Trel.append(T_rel.cpu().numpy())
            got_Tabs.append(T_abs.result())
    out[rank] = (np.concatenate(got_rec).tobytes(),
                 np.concatenate(got_Trel).tobytes() if got_Trel else b"",
                 np.concatenate(got_Tabs).tobytes() if got_Tabs else b"")
    run.close()
    dist.destroy_process_group()


def _single_rank(ctx, W, H, NF, F, blank, T0=None):
    import torch
    from droplet_visual_odometry_amd.stream import FrameStream
    from droplet_visual_odometry_amd.synth import MARKER_LEN
    frames, corners, K = _stream(W, H, F, blank)
    fs = FrameStream(W, H, K, nfeatures=NF, max_frames=F, ctx=ctx)
    fs.reset_pose(None, T0)
    rec = fs.process(torch.from_numpy(frames).cuda())
    dc = torch.from_numpy(corners).cuda()
    T_rel, T_abs = fs.pose_tail(dc[:-1], dc[1:], MARKER_LEN)
    fs.sync()
    out = rec.cpu().numpy().tobytes(), T_rel.cpu().numpy(), T_abs.cpu().numpy()
    fs.close()
    return out


def _check(gpu_ctx, out, ranks, W, H, NF, F, blank, T0=None):
    from droplet_visual_odometry_amd._native import PAIR_RECORD_DTYPE
    want_rec, want_Trel, want_Tabs = _single_rank(gpu_ctx, W, H, NF, F, blank, T0)
    st = np.frombuffer(want_rec, PAIR_RECORD_DTYPE)["status"]
    for b in blank:  # the blank frame's two pairs fail in the single-rank run too
        assert st[b - 1] != 0 and st[b] != 0
    for r in range(ranks):
        assert out[r][0] == want_rec, f"rank {r}: gathered records differ from the single-rank stream"
    np.testing.assert_array_equal(np.frombuffer(out[0][1]).reshape(-1, 4, 4), want_Trel)
    got_Tabs = np.frombuffer(out[0][2]).reshape(-1, 4, 4)
    # bit for bit (the host chain repeats the device chain's arithmetic), signed zeros included
    bad = [i for i in range(len(want_Tabs)) if got_Tabs[i].tobytes() != want_Tabs[i].tobytes()]
    assert not bad, f"rank 0 T_abs differs at pairs {bad}"


@pytest.mark.parametrize("W,H,NF,n_pairs,windows,blank", [
    (640, 480, 500, 6, 2, ()),
    (640, 480, 500, 5, 1, ()),
    # BASELINE configs[3] workload; frame 3 is rank 1's first frame, so pairs 2 (rank 0) and 3
    # (rank 1) fail and pair 4 triangulates against pair 1's P (rank 0); frame 6 fails the last
    # pair of window 0 and the first of window 1, so pair 7 uses pair 4's P from the carry
    (1280, 720, 2000, 6, 2, (3, 6)),
])
def test_sharded_stream_equals_single_rank(gpu_ctx, W, H, NF, n_pairs, windows, blank):
    import torch.multiprocessing as mp
    F = n_pairs * windows + 1
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), "gloo", W, H, NF, n_pairs, windows, blank, 1, out), nprocs=2, join=True)
    _check(gpu_ctx, out, 2, W, H, NF, F, blank)


def test_sharded_stream_reset_pose_non_identity(gpu_ctx):
    """ShardedStreamRunner.reset_pose seeds both halves of the split tail: every rank's P_prev and
    rank 0's host chain, so a non-identity T0 carries into T_abs as in one rank's pose tail."""
    import torch.multiprocessing as mp
    from droplet_visual_odometry_amd.transformations import euler_matrix
    T0 = euler_matrix(0.1, -0.2, 0.3)
    T0[:3, 3] = (0.5, -1.25, 2.0)
    n_pairs, windows = 5, 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), "gloo", W, H, NF, n_pairs, windows, (), 1, out, T0), nprocs=2, join=True)
    _check(gpu_ctx, out, 2, W, H, NF, n_pairs * windows + 1, (), T0)


@pytest.mark.parametrize("W,H,NF", [(640, 480, 500), (1280, 720, 2000)])
def test_sharded_rccl_path_two_slots_in_flight(gpu_ctx, W, H, NF):
    """The RCCL branch of the sharded loop (device all-gather, no host syncs):
    world size 1 on the box's one GPU, two streams with pipeline_depth()
    send-buffer slots each over fourteen windows, so every slot is rewritten
    while the previous windows' collectives and pose tails are still queued.  Any missing stream order (records read
    before written, a send buffer rewritten before its collective read it, the
    tail racing the gather) shows as a mismatch with the single-rank stream.
    Also at BASELINE configs[3]'s 1280x720 / 2000 features."""
    import torch.multiprocessing as mp
    n_pairs, windows, blank = 8, 14, (12,)  # more windows than streams x pipeline depth: slots reused
    F = n_pairs * windows + 1
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(1, _free_port(), "nccl", W, H, NF, n_pairs, windows, blank, 2, out), nprocs=1, join=True)
    _check(gpu_ctx, out, 1, W, H, NF, F, blank)


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


def test_host_chain_equals_device_chain(gpu_ctx):
    """dvo_pose_chain_host (rank 0's chain of a sharded stream) gives the device pose tail's T_abs
    byte for byte over 600 pairs of real T_rel, in two windows with the carry in between."""
    import ctypes
    import torch
    from conftest import synth_frames
    from droplet_visual_odometry_amd.stream import FrameStream
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    frames, K = synth_frames(320, 240, range(9))
    fs = FrameStream(320, 240, K, nfeatures=300, max_frames=9, ctx=gpu_ctx)
    fs.reset_pose()
    fs.process(torch.from_numpy(frames).cuda())
    dc = torch.from_numpy(np.stack([marker_corners(i, K) for i in range(9)])).cuda()
    T_rel, T_abs = fs.pose_tail(dc[:-1], dc[1:], MARKER_LEN)
    fs.sync()
    Tr = np.ascontiguousarray(np.tile(T_rel.cpu().numpy(), (75, 1, 1)))  # 600 pairs
    dev_abs = torch.empty((600, 4, 4), dtype=torch.float64, device="cuda")
    carry = torch.from_numpy(np.eye(4).reshape(16).copy()).cuda()
    gpu_ctx.check(gpu_ctx.lib.dvo_pose_chain(gpu_ctx.h, torch.from_numpy(Tr).cuda().data_ptr(), 600,
                                             carry.data_ptr(), dev_abs.data_ptr(), None))
    torch.cuda.synchronize()
    hc = np.eye(4).reshape(16).copy()
    out = np.empty((600, 4, 4))
    for a, b in ((0, 250), (250, 600)):
        part = np.ascontiguousarray(Tr[a:b])
        o = np.empty_like(part)
        assert gpu_ctx.lib.dvo_pose_chain_host(part.ctypes.data, b - a, hc.ctypes.data, o.ctypes.data) == 0
        out[a:b] = o
    assert out.tobytes() == dev_abs.cpu().numpy().tobytes()
    assert hc.tobytes() == carry.cpu().numpy().tobytes()
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
