"""The reference's own schedule on the device (dvo_stream_process_pairs):
visual_odometry_calculations re-detects BOTH frames of every pair
(visual_odometry_v3.py:387-392), so pair p is frames 2p, 2p+1 detected on
their own.  Detection is a function of the frame alone, so every record, match
list and pose must equal the streaming schedule's (each frame detected once)
bit for bit, and the oracle's (which re-detects both frames) too."""
import numpy as np
import pytest

from conftest import synth_frames

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W,H,NF,n", [(640, 480, 500, 5), (1280, 720, 2000, 5), (320, 240, 300, 301)])
def test_pairs_schedule_equals_stream(gpu_ctx, W, H, NF, n):
    """n = 301: both schedules detect in frame groups (301 and 600 frames, csrc/orb.hip launch_orb)."""
    import torch
    from droplet_visual_odometry_amd.stream import FrameStream
    frames, K = synth_frames(W, H, range(n))
    dev = torch.from_numpy(frames).cuda()
    paired = torch.stack([dev[i + j] for i in range(n - 1) for j in (0, 1)]).contiguous()
    a = FrameStream(W, H, K, nfeatures=NF, max_frames=n, ctx=gpu_ctx)
    b = FrameStream(W, H, K, nfeatures=NF, max_frames=2 * (n - 1), ctx=gpu_ctx)
    ra = a.process(dev)
    rb = b.process_pairs(paired)
    a.sync()
    b.sync()
    A, B = FrameStream.records_numpy(ra, n - 1), FrameStream.records_numpy(rb, n - 1)
    for k in A.dtype.names:
        bad = np.nonzero(~np.all((A[k] == B[k]).reshape(n - 1, -1), axis=1))[0]
        assert len(bad) == 0, f"field {k} differs at pairs {bad[:10]}"
    np.testing.assert_array_equal(ra.cpu().numpy(), rb.cpu().numpy())
    for p in list(range(min(n - 1, 4))) + [n - 2]:
        np.testing.assert_array_equal(a.matches(p), b.matches(p))
        ka, da = a.features(p + 1)
        kb, db = b.features(2 * p + 1)
        np.testing.assert_array_equal(ka.view(np.uint8), kb.view(np.uint8))
        np.testing.assert_array_equal(da, db)
    a.close()
    b.close()


def test_pairs_schedule_pose_tail_and_oracle(gpu_ctx, oracle_mod):
    """R, t of the paired schedule equal the oracle's re-detecting pair_pose;
    the device pose tail after process_pairs equals the one after process."""
    import torch
    from droplet_visual_odometry_amd.stream import FrameStream
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    n = 4
    frames, K = synth_frames(640, 480, range(n))
    corners = np.stack([marker_corners(i, K) for i in range(n)])
    dc = torch.from_numpy(corners).cuda()
    dev = torch.from_numpy(frames).cuda()
    paired = torch.stack([dev[i + j] for i in range(n - 1) for j in (0, 1)]).contiguous()
    fs = FrameStream(640, 480, K, nfeatures=500, max_frames=2 * (n - 1), ctx=gpu_ctx)
    fs.reset_pose()
    rec = fs.process_pairs(paired)
    Tp = fs.pose_tail(dc[:-1], dc[1:], MARKER_LEN)
    fs.sync()  # the tail ran on the library stream: read it before the next call reuses the carry
    Tp = [t.clone() for t in Tp]
    fs.reset_pose()
    fs.process(dev)
    Ts = fs.pose_tail(dc[:-1], dc[1:], MARKER_LEN)
    fs.sync()
    for x, y in zip(Tp, Ts):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())
    recs = FrameStream.records_numpy(rec, n - 1)
    for p in range(n - 1):
        ref = oracle_mod.pair_pose(frames[p], frames[p + 1], K, 500)  # both frames detected
        assert recs[p]["status"] == 0
        assert recs[p]["n_matches"] == len(ref["q"])
        np.testing.assert_array_equal(recs[p]["R"].reshape(3, 3), ref["R"])
        np.testing.assert_array_equal(recs[p]["t"], ref["t_unit"].ravel())
    fs.close()


def test_pairs_schedule_argument_checks(gpu_ctx):
    import torch
    from droplet_visual_odometry_amd._native import DVOError
    from droplet_visual_odometry_amd.stream import FrameStream
    K = np.array([[500.0, 0, 320], [0, 500, 240], [0, 0, 1]])
    fs = FrameStream(640, 480, K, nfeatures=500, max_frames=4, ctx=gpu_ctx)
    with pytest.raises(ValueError):
        fs.process_pairs(torch.zeros((3, 480, 640), dtype=torch.uint8, device="cuda"))
    with pytest.raises(DVOError):  # 3 pairs = 6 frames > max_frames
        fs.process_pairs(torch.zeros((6, 480, 640), dtype=torch.uint8, device="cuda"))
    fs.close()
