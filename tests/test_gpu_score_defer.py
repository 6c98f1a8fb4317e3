"""The RANSAC score's deferred f64 Sampson tests (geometry.hip
ransac_score_kernel): points the single-precision bounds
leave undecided are listed per block in LDS and tested in f64 after the last
chunk; a full list falls back to the inline test.  A camera whose focal
length is tiny makes every normalised coordinate large (> 1e6: outside
SampsonF32's range), so the f32 bounds leave every (model, point) pair
undecided and both the list and its overflow run.
E, mask, R, t bit-exact against the oracle (visual_odometry_v3.py:297-306)."""
import numpy as np
import pytest

from conftest import synth_frames

pytestmark = pytest.mark.gpu


def test_find_essential_all_undecided(gpu_ctx, oracle_mod):
    from droplet_visual_odometry_amd import ops
    from droplet_visual_odometry_amd._native import DVOError
    from test_gpu_configs import _correspondences
    p1, p2, K0 = _correspondences(11, 1200, 0.5)
    models = 0
    for f in (1e-4, 3e-5, 1e-5):
        K = K0.copy()
        K[0, 0] = K[1, 1] = f
        for max_iters in (65, 300):
            Eo, mo, io = oracle_mod.find_essential(p1, p2, K, max_iters=max_iters)
            if Eo is None:
                with pytest.raises(DVOError):
                    ops.find_essential_mat(p1, p2, K, max_iters=max_iters, ctx=gpu_ctx)
                continue
            models += 1
            E, mask = ops.find_essential_mat(p1, p2, K, max_iters=max_iters, ctx=gpu_ctx)
            np.testing.assert_array_equal(E, Eo)
            np.testing.assert_array_equal(mask.ravel(), mo.ravel())
    assert models > 0, "no case reached a model: the f64 inlier path is not exercised"


def test_stream_all_undecided(gpu_ctx, oracle_mod):
    """The batched path (16 hypotheses per score block) with a tiny focal
    length: records bit-identical to the oracle's pair_pose."""
    import torch
    from droplet_visual_odometry_amd.stream import FrameStream
    frames, K = synth_frames(640, 480, range(3))
    K = K.copy()
    K[0, 0] = K[1, 1] = 1e-4
    fs = FrameStream(640, 480, K, nfeatures=500, max_frames=3, ctx=gpu_ctx)
    rec = fs.process(torch.from_numpy(frames).cuda())
    fs.sync()
    recs = FrameStream.records_numpy(rec, 2)
    kp = None
    for p in range(2):
        ref = oracle_mod.pair_pose(frames[p], frames[p + 1], K, 500, kp_prev=kp)
        kp = (ref["kp_cur"], ref["desc_cur"])
        assert recs[p]["n_matches"] == len(ref["q"])
        if ref["R"] is None:
            assert recs[p]["status"] != 0
            continue
        assert recs[p]["status"] == 0
        np.testing.assert_array_equal(recs[p]["R"].reshape(3, 3), ref["R"])
        np.testing.assert_array_equal(recs[p]["t"], ref["t_unit"].ravel())
    fs.close()
