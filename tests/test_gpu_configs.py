"""BASELINE.json configurations on the GPU, bit-exact against the oracle:

  configs[1]  640x480 stream, 1000 ORB features (C2)
  configs[4]  1920x1080 stream, 4000 features, 5-point RANSAC at maxIters 4096 (C5)

findEssentialMat's iteration count is adaptive (RANSACUpdateNumIters,
visual_odometry_v3.py:297-300 -> OpenCV's RANSACPointSetRegistrator): a pair
with a low inlier ratio runs past the replay chunk (1024 hypotheses) and up to
the 4096 cap, which exercises every buffer the stream sizes by max_iters
(api.cpp: models, subsets, gscr, fprec, dk_list) and the second RANSAC round.
"""
import numpy as np
import pytest

from conftest import synth_frames

pytestmark = pytest.mark.gpu


def _check_stream(fs, frames, K, n, order, oracle_mod, max_iters):
    import torch
    from droplet_visual_odometry_amd.stream import FrameStream
    seq = frames[order]
    rec = fs.process(torch.from_numpy(np.ascontiguousarray(seq)).cuda())
    fs.sync()
    recs = FrameStream.records_numpy(rec, len(order) - 1)
    iters = []
    kp_prev = None
    for i in range(len(order) - 1):
        ref = oracle_mod.pair_pose(seq[i], seq[i + 1], K, n, max_iters=max_iters, kp_prev=kp_prev)
        kp_prev = (ref["kp_cur"], ref["desc_cur"])
        kg, dg = fs.features(i + 1)
        np.testing.assert_array_equal(kg.view(np.uint8), ref["kp_cur"].view(np.uint8))
        np.testing.assert_array_equal(dg, ref["desc_cur"])
        mg = fs.matches(i)
        np.testing.assert_array_equal(mg["queryIdx"], ref["q"])
        np.testing.assert_array_equal(mg["trainIdx"], ref["t"])
        r = recs[i]
        assert r["status"] == 0
        assert r["ransac_iters"] == ref["iters"], (i, r["ransac_iters"], ref["iters"])
        assert r["n_inliers"] == int(ref["mask"].sum())
        np.testing.assert_array_equal(r["E"].reshape(3, 3), ref["E"])
        np.testing.assert_array_equal(r["R"].reshape(3, 3), ref["R"])
        np.testing.assert_array_equal(r["t"], ref["t_unit"].ravel())
        assert r["n_good"] == ref["good"]
        iters.append(int(r["ransac_iters"]))
    return iters


def test_c2_640x480_1000_features(gpu_ctx, oracle_mod):
    """configs[1]: three consecutive pairs of the 640x480 stream at N = 1000."""
    from droplet_visual_odometry_amd.stream import FrameStream
    frames, K = synth_frames(640, 480, range(4))
    fs = FrameStream(640, 480, K, nfeatures=1000, max_frames=4, ctx=gpu_ctx)
    _check_stream(fs, frames, K, 1000, [0, 1, 2, 3], oracle_mod, 1000)
    fs.close()


def test_c5_1920x1080_4000_features_4096_hypotheses(gpu_ctx, oracle_mod):
    """configs[4]: 1920x1080, N = 4000, maxIters = 4096.  Frames 0-3 are
    consecutive (high inlier ratio, tens of iterations); the jump 3 -> 9 is a
    wide-baseline pair whose inlier ratio drives RANSAC to the 4096 cap, past
    the 1000 default and the 1024-hypothesis replay chunk."""
    from droplet_visual_odometry_amd.stream import FrameStream
    idx = [0, 1, 2, 3, 9, 10]
    frames, K = synth_frames(1920, 1080, idx)
    fs = FrameStream(1920, 1080, K, nfeatures=4000, max_frames=len(idx), max_iters=4096, ctx=gpu_ctx)
    iters = _check_stream(fs, frames, K, 4000, list(range(len(idx))), oracle_mod, 4096)
    assert max(iters) > 1024, iters
    fs.close()


def _correspondences(seed, m, inlier_frac):
    """Two views of a random 3-D cloud (1920x1080 intrinsics, 0.3 px noise),
    with 1 - inlier_frac of the second view's points replaced by uniform
    outliers; float32-rounded as KeyPoint_convert output is (v3:355)."""
    rng = np.random.default_rng(seed)
    f = 1820.433
    K = np.array([[f, 0, 960], [0, f, 540], [0, 0, 1.0]])
    X = np.c_[rng.uniform(-2, 2, (m, 2)), rng.uniform(3, 8, m)]
    a = 0.05
    R = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
    X2 = X @ R.T + np.array([0.3, 0.02, 0.1])
    p1 = X[:, :2] / X[:, 2:] * f + [960, 540]
    p2 = X2[:, :2] / X2[:, 2:] * f + [960, 540]
    p1 += rng.normal(0, 0.3, p1.shape)
    p2 += rng.normal(0, 0.3, p2.shape)
    nout = int(m * (1 - inlier_frac))
    out = rng.choice(m, nout, replace=False)
    p2[out] = rng.uniform([0, 0], [1920, 1080], (nout, 2))
    return p1.astype(np.float32).astype(np.float64), p2.astype(np.float32).astype(np.float64), K


@pytest.mark.parametrize("inlier_frac,max_iters,regime", [
    (0.35, 4096, "adaptive"),    # oracle: 1972 iterations
    (0.30, 4096, "adaptive"),    # oracle: 3524 iterations
    (0.25, 4096, "cap"),         # 4096
    (0.25, 1025, "cap"),         # one hypothesis past the replay chunk
    (0.25, 2048, "cap"),
    (0.25, 65, "cap"),           # round 1 (64) + one
])
def test_find_essential_past_the_replay_chunk(gpu_ctx, oracle_mod, inlier_frac, max_iters, regime):
    """findEssentialMat on 1500 correspondences whose inlier ratio puts the
    adaptive iteration count between 1024 and 4096 (or at the cap): E and the
    inlier mask bit-exact against the oracle."""
    from droplet_visual_odometry_amd import ops
    p1, p2, K = _correspondences(5, 1500, inlier_frac)
    Eo, mo, io = oracle_mod.find_essential(p1, p2, K, max_iters=max_iters)
    if regime == "adaptive":
        assert 1024 < io < max_iters, io
    else:
        assert io == max_iters, io
    E, mask = ops.find_essential_mat(p1, p2, K, max_iters=max_iters, ctx=gpu_ctx)
    np.testing.assert_array_equal(E, Eo)
    np.testing.assert_array_equal(mask.ravel(), mo.ravel())
