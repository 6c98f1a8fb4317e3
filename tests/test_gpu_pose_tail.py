"""Device pose tail (dvo_stream_pose_tail) vs the host restatement of
visual_odometry_v3.py:309-345 / :367 (oracle.pose_tail), chained across two
batches so the device carry (P_prev, T_abs) is exercised.

Tolerance: the tail is float64 arithmetic with libm atan2/sin/cos/sqrt on both
sides (ocml on the device, glibc on the host, each <= 1 ulp off) and numpy's
3x3 / 4x4 products; 1e-9 relative on every entry of T_rel and T_abs."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_pose_tail_two_batches(gpu_ctx, oracle_mod):
    import torch
    from conftest import synth_frames
    from droplet_visual_odometry_amd.stream import FrameStream
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    frames, K = synth_frames(640, 480, range(7))
    corners = np.stack([marker_corners(i, K) for i in range(7)])
    fs = FrameStream(640, 480, K, nfeatures=500, max_frames=4, ctx=gpu_ctx)
    fs.reset_pose()
    P = K @ np.hstack((np.eye(3), np.zeros((3, 1))))
    T = np.eye(4)
    dc = torch.from_numpy(corners).cuda()
    for start in (0, 3):
        dev = torch.from_numpy(frames[start:start + 4]).cuda()
        rec = fs.process(dev)
        T_rel, T_abs = fs.pose_tail(dc[start:start + 3], dc[start + 1:start + 4], MARKER_LEN)
        fs.sync()
        recs = FrameStream.records_numpy(rec, 3)
        T_rel, T_abs = T_rel.cpu().numpy(), T_abs.cpu().numpy()
        for p in range(3):
            r = recs[p]
            assert r["status"] == 0
            P, Tr, T = oracle_mod.pose_tail(K, r["R"].reshape(3, 3), r["t"], corners[start + p],
                                            corners[start + p + 1], MARKER_LEN, P, T)
            np.testing.assert_allclose(T_rel[p], Tr, rtol=1e-9, atol=1e-12)
            np.testing.assert_allclose(T_abs[p], T, rtol=1e-9, atol=1e-12)
    fs.close()


def test_pose_tail_requires_process(gpu_ctx):
    import torch
    from droplet_visual_odometry_amd._native import DVOError
    from droplet_visual_odometry_amd.stream import FrameStream
    K = np.array([[500.0, 0, 320], [0, 500, 240], [0, 0, 1]])
    fs = FrameStream(640, 480, K, nfeatures=500, max_frames=2, ctx=gpu_ctx)
    c = torch.zeros((1, 4, 2), dtype=torch.float64, device="cuda")
    with pytest.raises(DVOError):
        fs.pose_tail(c, c, 0.1)
    fs.close()


def test_two_streams_share_one_pose_chain(gpu_ctx):
    """Batches alternating between two dvo_streams (own HIP streams, overlapping
    on the device) with a shared carry give the single-stream pose chain."""
    import torch
    from conftest import synth_frames
    from droplet_visual_odometry_amd.stream import FrameStream
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    frames, K = synth_frames(640, 480, range(7))
    dev = torch.from_numpy(frames).cuda()
    dc = torch.from_numpy(np.stack([marker_corners(i, K) for i in range(7)])).cuda()
    ref = FrameStream(640, 480, K, nfeatures=500, max_frames=4, ctx=gpu_ctx)
    ref.reset_pose()
    want = []
    for start in (0, 3):
        ref.process(dev[start:start + 4])
        want.append(ref.pose_tail(dc[start:start + 3], dc[start + 1:start + 4], MARKER_LEN)[1])
    ref.sync()
    a = FrameStream(640, 480, K, nfeatures=500, max_frames=4, ctx=gpu_ctx)
    b = FrameStream(640, 480, K, nfeatures=500, max_frames=4, ctx=gpu_ctx)
    b.share_pose(a)
    a.reset_pose()
    got = []
    for fs, start in ((a, 0), (b, 3)):
        fs.process(dev[start:start + 4])
        got.append(fs.pose_tail(dc[start:start + 3], dc[start + 1:start + 4], MARKER_LEN)[1])
    a.sync()
    b.sync()
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g.cpu().numpy(), w.cpu().numpy())
    for fs in (ref, a, b):
        fs.close()


def test_pose_tail_from_stag_messages(gpu_ctx, oracle_mod):
    """Corners arriving as StagMarkers-style messages (traj_eval_ground_truth.py:303-311),
    packed by marker_corner_batch, drive the same device tail as raw arrays."""
    import os
    import sys
    from types import SimpleNamespace as NS
    import torch
    from conftest import ROOT, synth_frames
    sys.path.insert(0, os.path.join(ROOT, "droplet_visual_odometry_amd", "dropin"))
    import marker_corners as mc
    from droplet_visual_odometry_amd.stream import FrameStream
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    frames, K = synth_frames(640, 480, range(4))
    corners = [marker_corners(i, K) for i in range(4)]
    msgs = [NS(markers=[NS(id=0, corners=[NS(x=x, y=y) for x, y in c])]) for c in corners]
    dc = mc.marker_corner_batch(msgs, device="cuda")
    fs = FrameStream(640, 480, K, nfeatures=500, max_frames=4, ctx=gpu_ctx)
    fs.reset_pose()
    rec = fs.process(torch.from_numpy(frames).cuda())
    T_rel, T_abs = fs.pose_tail(dc[:-1], dc[1:], MARKER_LEN)
    fs.sync()
    recs = FrameStream.records_numpy(rec, 3)
    P, T = K @ np.hstack((np.eye(3), np.zeros((3, 1)))), np.eye(4)
    T_abs = T_abs.cpu().numpy()
    for p in range(3):
        assert recs[p]["status"] == 0
        P, _, T = oracle_mod.pose_tail(K, recs[p]["R"].reshape(3, 3), recs[p]["t"], corners[p], corners[p + 1],
                                       MARKER_LEN, P, T)
        np.testing.assert_allclose(T_abs[p], T, rtol=1e-9, atol=1e-12)
    fs.close()


def test_pose_tail_after_caller_dropped_records(gpu_ctx):
    """process() allocates the records; the caller drops them and allocates on
    torch's stream before pose_tail.  The stream keeps the last records alive
    (the tail reads them), so T_rel/T_abs equal a run that held them."""
    import gc
    import torch
    from conftest import synth_frames
    from droplet_visual_odometry_amd.stream import FrameStream
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    frames, K = synth_frames(640, 480, range(4))
    dev = torch.from_numpy(frames).cuda()
    dc = torch.from_numpy(np.stack([marker_corners(i, K) for i in range(4)])).cuda()
    fs = FrameStream(640, 480, K, nfeatures=500, max_frames=4, ctx=gpu_ctx)
    fs.reset_pose()
    kept = fs.process(dev)
    want = fs.pose_tail(dc[:-1], dc[1:], MARKER_LEN)
    fs.sync()
    want = [t.clone() for t in want]
    del kept
    fs.reset_pose()
    fs.process(dev)  # result dropped at once
    gc.collect()
    junk = [torch.full((4096,), 255, dtype=torch.uint8, device="cuda") for _ in range(16)]  # reuse freed blocks
    got = fs.pose_tail(dc[:-1], dc[1:], MARKER_LEN)
    junk += [torch.full((4096,), 255, dtype=torch.uint8, device="cuda") for _ in range(16)]
    fs.sync()
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g.cpu().numpy(), w.cpu().numpy())
    fs.close()
