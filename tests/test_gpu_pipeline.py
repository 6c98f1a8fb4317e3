"""Pipelined batches (dvo_stream_submit, include/dvo.h): findEssentialMat's
RANSAC loop (RANSACPointSetRegistrator::run, visual_odometry_v3.py:297) runs in
rounds of hypotheses; a submit runs ONE merged round in which each of the last
pipeline_depth() batches takes its next round, and retires the batch whose last
round ran.  Whatever the schedule, every record must equal the one-batch-at-a-time
dvo_stream_process's byte for byte, the pose tail over retired batches must equal
the per-batch tail, and batches must retire in submission order."""
import numpy as np
import pytest

from conftest import synth_frames

pytestmark = pytest.mark.gpu


def _stream(W, H, n, blank=()):
    from droplet_visual_odometry_amd.synth import marker_corners
    frames, K = synth_frames(W, H, range(n))
    frames = frames.copy()
    corners = [marker_corners(i, K) for i in range(n)]
    for b in blank:
        frames[b] = 90
        corners[b] = corners[b - 1]
    return frames, np.stack(corners), K


@pytest.mark.parametrize("W,H,NF,sizes,blank", [
    (640, 480, 500, [5, 5, 5, 5, 5, 5, 5, 3], ()),          # more batches than the pipeline holds, a short last one
    (320, 240, 300, [9, 2, 9, 9, 4, 9, 9], (6, 14)),        # featureless frames: failing pairs
    (1280, 720, 2000, [4, 4, 4, 4, 4, 4], ()),
])
def test_submit_equals_process(gpu_ctx, W, H, NF, sizes, blank):
    import torch
    from droplet_visual_odometry_amd.stream import FrameStream
    from droplet_visual_odometry_amd.synth import MARKER_LEN
    D = FrameStream.pipeline_depth()
    assert D >= 2
    # batches of a stream: batch b = frames [s_b, s_b + sizes[b]), consecutive batches share a frame
    starts = np.concatenate([[0], np.cumsum(np.array(sizes) - 1)])[:-1]
    n = int(starts[-1] + sizes[-1])
    frames, corners, K = _stream(W, H, n, blank)
    dev = torch.from_numpy(frames).cuda()
    dc = torch.from_numpy(corners).cuda()
    F = max(sizes)
    a = FrameStream(W, H, K, nfeatures=NF, max_frames=F, ctx=gpu_ctx)
    b = FrameStream(W, H, K, nfeatures=NF, max_frames=F, ctx=gpu_ctx)
    a.reset_pose()
    b.reset_pose()
    want, want_T = [], []
    for s0, m in zip(starts, sizes):
        r = a.process(dev[s0:s0 + m])
        Tr, Ta = a.pose_tail(dc[s0:s0 + m - 1], dc[s0 + 1:s0 + m], MARKER_LEN)
        a.sync()
        want.append(FrameStream.records_numpy(r, m - 1))
        want_T.append((Tr.cpu().numpy(), Ta.cpu().numpy()))
    recs = [b.new_records(m - 1) for m in sizes]
    torch.cuda.synchronize()
    order, got_T = [], []

    def tails(retired):
        for rec, pairs in retired:
            i = next(j for j, r in enumerate(recs) if r.data_ptr() == rec.data_ptr())
            assert pairs == sizes[i] - 1
            s0 = int(starts[i])
            Tr = torch.empty((pairs, 4, 4), dtype=torch.float64, device=dev.device)
            Ta = torch.empty_like(Tr)
            b.pose_tail_batch(rec, pairs, dc[s0:s0 + pairs], dc[s0 + 1:s0 + pairs + 1], MARKER_LEN, Tr, Ta)
            order.append(i)
            got_T.append((Tr, Ta))

    for i, (s0, m) in enumerate(zip(starts, sizes)):
        ret = b.submit(dev[s0:s0 + m], recs[i], wait_torch=False)
        ptrs = [r.data_ptr() for r in recs]
        assert [ptrs.index(x.data_ptr()) for x, _ in ret] == ([i - (D - 1)] if i >= D - 1 else [])
        tails(ret)
    tails(b.drain())
    b.sync()
    assert order == list(range(len(sizes)))
    for i, m in enumerate(sizes):
        got = FrameStream.records_numpy(recs[i], m - 1)
        for k in got.dtype.names:
            bad = np.nonzero(~np.all((got[k] == want[i][k]).reshape(m - 1, -1), axis=1))[0]
            assert len(bad) == 0, f"batch {i} field {k} differs at pairs {bad[:10]}"
        np.testing.assert_array_equal(got_T[i][0].cpu().numpy(), want_T[i][0])
        np.testing.assert_array_equal(got_T[i][1].cpu().numpy(), want_T[i][1])
    if blank:
        allrec = np.concatenate(want)
        assert np.any(allrec["status"] != 0)
    a.close()
    b.close()


def test_process_drains_pending_submits(gpu_ctx):
    """A dvo_stream_process after pipelined submits retires them first (their records complete),
    and the stream-pair path refuses to run while batches are pending."""
    import torch
    from droplet_visual_odometry_amd._native import DVOError
    from droplet_visual_odometry_amd.stream import FrameStream
    frames, _, K = _stream(640, 480, 9)
    dev = torch.from_numpy(frames).cuda()
    ref = FrameStream(640, 480, K, nfeatures=500, max_frames=5, ctx=gpu_ctx)
    fs = FrameStream(640, 480, K, nfeatures=500, max_frames=5, ctx=gpu_ctx)
    want = []
    for s0 in (0, 4):
        r = ref.process(dev[s0:s0 + 5])
        ref.sync()  # the records are written on the library's stream
        want.append(FrameStream.records_numpy(r, 4))
    r0 = fs.new_records(4)
    torch.cuda.synchronize()
    assert fs.submit(dev[0:5], r0, wait_torch=False) == []
    r1 = fs.process(dev[4:9])
    fs.sync()
    for name, r, w in (("r0", r0, want[0]), ("r1", r1, want[1])):
        got = FrameStream.records_numpy(r, 4)
        assert [k for k in got.dtype.names if not np.array_equal(got[k], w[k])] == [], \
            (name, got["n_matches"], w["n_matches"], got["ransac_iters"], w["ransac_iters"], got["n_hypotheses"],
             w["n_hypotheses"], got["status"], w["status"])
    r2 = fs.new_records(4)
    torch.cuda.synchronize()
    fs.submit(dev[0:5], r2, wait_torch=False)
    from droplet_visual_odometry_amd._native import PAIR_RECORD_DTYPE
    host_rec = np.zeros(1, PAIR_RECORD_DTYPE)
    with pytest.raises(DVOError):
        fs.ctx.check(fs.ctx.lib.dvo_stream_pair(fs.h, frames[0].ctypes.data, frames[1].ctypes.data, 640, 0,
                                                host_rec.ctypes.data))
    fs.drain()
    fs.sync()
    assert FrameStream.records_numpy(r2, 4).tobytes() == want[0].tobytes()
    ref.close()
    fs.close()


def test_submit_pairs_equals_process_pairs(gpu_ctx):
    import torch
    from droplet_visual_odometry_amd.stream import FrameStream
    frames, _, K = _stream(640, 480, 12)
    dev = torch.from_numpy(frames).cuda()
    paired = [torch.stack([dev[i + j] for i in range(s, s + 3) for j in (0, 1)]).contiguous() for s in (0, 3, 6, 8)]
    a = FrameStream(640, 480, K, nfeatures=500, max_frames=6, ctx=gpu_ctx)
    b = FrameStream(640, 480, K, nfeatures=500, max_frames=6, ctx=gpu_ctx)
    want = []
    for p in paired:
        r = a.process_pairs(p)
        a.sync()
        want.append(FrameStream.records_numpy(r, 3))
    recs = [b.new_records(3) for _ in paired]
    torch.cuda.synchronize()
    for p, r in zip(paired, recs):
        b.submit_pairs(p, r, wait_torch=False)
    b.drain()
    b.sync()
    for w, r in zip(want, recs):
        assert FrameStream.records_numpy(r, 3).tobytes() == w.tobytes()
    a.close()
    b.close()
