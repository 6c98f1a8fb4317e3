"""Edge cases on the GPU vs the oracle: blank and tiny frames (levels below the
31-px ORB border produce no features), odd sizes, few matches, detect-only
stream calls, the maximum nfeatures, the larger BASELINE configurations."""
import numpy as np
import pytest

from conftest import synth_frames

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wh", [(8, 8), (40, 30), (63, 63), (64, 64), (100, 80), (161, 97), (333, 211)])
def test_detect_small_and_odd_sizes(gpu_ctx, oracle_mod, wh):
    from droplet_visual_odometry_amd import ops
    w, h = wh
    rng = np.random.default_rng(w * 1000 + h)
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    img = np.ascontiguousarray(np.clip(img.astype(np.int32) // 2 + np.add.outer(np.arange(h), np.arange(w)) % 128,
                                       0, 255).astype(np.uint8))
    kg, dg = ops.detect_and_compute(img, 500, ctx=gpu_ctx)
    ko, do = oracle_mod.detect_and_compute(img, 500)
    assert len(kg) == len(ko)
    np.testing.assert_array_equal(kg.view(np.uint8), ko.view(np.uint8))
    np.testing.assert_array_equal(dg, do)


def test_blank_frame_has_no_features(gpu_ctx, oracle_mod):
    from droplet_visual_odometry_amd import ops
    img = np.full((480, 640), 128, np.uint8)
    kg, _ = ops.detect_and_compute(img, 500, ctx=gpu_ctx)
    ko, _ = oracle_mod.detect_and_compute(img, 500)
    assert len(kg) == len(ko) == 0


def test_stream_blank_pair_status(gpu_ctx):
    import torch
    from droplet_visual_odometry_amd._native import DVO_ENOFEAT
    from droplet_visual_odometry_amd.stream import FrameStream
    frames, K = synth_frames(640, 480, range(2))
    blank = np.full((480, 640), 77, np.uint8)
    seq = np.stack([frames[0], blank, frames[1]])
    fs = FrameStream(640, 480, K, nfeatures=500, max_frames=3, ctx=gpu_ctx)
    rec = fs.process(torch.from_numpy(seq).cuda())
    fs.sync()
    r = FrameStream.records_numpy(rec, 2)
    assert r["status"][0] == DVO_ENOFEAT and r["status"][1] == DVO_ENOFEAT
    assert r["n_kp_cur"][0] == 0 and r["n_kp_prev"][1] == 0
    fs.close()


def test_stream_single_frame_detect_only(gpu_ctx, oracle_mod):
    import torch
    from droplet_visual_odometry_amd.stream import FrameStream
    frames, K = synth_frames(640, 480, range(1))
    fs = FrameStream(640, 480, K, nfeatures=500, max_frames=2, ctx=gpu_ctx)
    fs.process(torch.from_numpy(frames[:1]).cuda())
    fs.sync()
    kg, dg = fs.features(0)
    ko, do = oracle_mod.detect_and_compute(frames[0], 500)
    np.testing.assert_array_equal(kg.view(np.uint8), ko.view(np.uint8))
    np.testing.assert_array_equal(dg, do)
    fs.close()


@pytest.mark.parametrize("m", [0, 4, 5, 6, 9])
def test_few_correspondences(gpu_ctx, oracle_mod, m):
    from droplet_visual_odometry_amd import ops
    from droplet_visual_odometry_amd._native import DVOError
    rng = np.random.default_rng(m)
    K = np.array([[500.0, 0, 320], [0, 500, 240], [0, 0, 1]])
    X = np.c_[rng.uniform(-1, 1, (m, 2)), rng.uniform(3, 6, m)]
    p1 = X[:, :2] / X[:, 2:] * 500 + [320, 240]
    X2 = X - [0.5, 0.0, 0.0]
    p2 = X2[:, :2] / X2[:, 2:] * 500 + [320, 240]
    Eo, mo, io = oracle_mod.find_essential(p1, p2, K)
    if m < 5:
        assert Eo is None
        with pytest.raises(DVOError):
            ops.find_essential_mat(p1, p2, K, ctx=gpu_ctx)
        return
    E, mask = ops.find_essential_mat(p1, p2, K, ctx=gpu_ctx)
    np.testing.assert_array_equal(E, Eo)
    np.testing.assert_array_equal(mask.ravel(), mo.ravel())


def test_max_nfeatures(gpu_ctx, oracle_mod):
    from droplet_visual_odometry_amd import ops
    frames, _ = synth_frames(1280, 720, range(1))
    kg, dg = ops.detect_and_compute(frames[0], 7680, ctx=gpu_ctx)
    ko, do = oracle_mod.detect_and_compute(frames[0], 7680)
    np.testing.assert_array_equal(kg.view(np.uint8), ko.view(np.uint8))
    np.testing.assert_array_equal(dg, do)


@pytest.mark.parametrize("w,h,n", [(1280, 720, 2000), (1920, 1080, 4000)])
def test_stream_baseline_configs(gpu_ctx, oracle_mod, w, h, n):
    """BASELINE.json configs[1] / configs[2] sizes, three pairs each, bit-exact."""
    import torch
    from droplet_visual_odometry_amd.stream import FrameStream
    frames, K = synth_frames(w, h, range(4))
    fs = FrameStream(w, h, K, nfeatures=n, max_frames=4, ctx=gpu_ctx)
    rec = fs.process(torch.from_numpy(frames).cuda())
    fs.sync()
    recs = FrameStream.records_numpy(rec, 3)
    kp_prev = None
    for i in range(3):
        ref = oracle_mod.pair_pose(frames[i], frames[i + 1], K, n, kp_prev=kp_prev)
        kp_prev = (ref["kp_cur"], ref["desc_cur"])
        kg, dg = fs.features(i + 1)
        np.testing.assert_array_equal(kg.view(np.uint8), ref["kp_cur"].view(np.uint8))
        np.testing.assert_array_equal(dg, ref["desc_cur"])
        mg = fs.matches(i)
        np.testing.assert_array_equal(mg["queryIdx"], ref["q"])
        np.testing.assert_array_equal(mg["trainIdx"], ref["t"])
        r = recs[i]
        assert r["status"] == 0 and r["ransac_iters"] == ref["iters"]
        np.testing.assert_array_equal(r["E"].reshape(3, 3), ref["E"])
        np.testing.assert_array_equal(r["R"].reshape(3, 3), ref["R"])
        np.testing.assert_array_equal(r["t"], ref["t_unit"].ravel())
        assert r["n_good"] == ref["good"]
    fs.close()


def test_golden_fixture_on_gpu(gpu_ctx):
    """The committed 320x240 golden pair (tests/golden/pair_320x240.npz)."""
    import os
    from droplet_visual_odometry_amd import ops
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "pair_320x240.npz"))
    nf = int(g["nfeatures"])
    for i, key in enumerate(("kp0", "kp1")):
        kg, dg = ops.detect_and_compute(g["frames"][i], nf, ctx=gpu_ctx)
        np.testing.assert_array_equal(kg.view(np.uint8).ravel(), g[key].view(np.uint8).ravel())
        np.testing.assert_array_equal(dg, g["desc0" if i == 0 else "desc1"])
    m = ops.bf_match(g["desc0"], g["desc1"], 1, ctx=gpu_ctx)
    order = np.argsort(m["distance"], kind="stable")
    np.testing.assert_array_equal(m["queryIdx"][order], g["q"])
    np.testing.assert_array_equal(m["trainIdx"][order], g["t"])
    E, mask = ops.find_essential_mat(g["p1"], g["p2"], g["K"], ctx=gpu_ctx)
    np.testing.assert_array_equal(E, g["E"])
    good, R, t, _ = ops.recover_pose(E, g["p1"], g["p2"], g["K"], ctx=gpu_ctx)  # v3:303: no mask
    np.testing.assert_array_equal(R, g["R"])
    np.testing.assert_array_equal(t.reshape(3, 1), g["t_unit"])
    assert good == int(g["good"])


def _degenerate_sets():
    rng = np.random.default_rng(7)
    K = np.array([[500.0, 0, 320], [0, 500, 240], [0, 0, 1]])
    X = np.c_[rng.uniform(-1, 1, (30, 2)), rng.uniform(3, 6, 30)]
    p1 = X[:, :2] / X[:, 2:] * 500 + [320, 240]
    X2 = X - [0.3, 0.1, 0.0]
    p2 = X2[:, :2] / X2[:, 2:] * 500 + [320, 240]
    line = np.c_[np.linspace(100, 500, 30), np.linspace(50, 400, 30)]
    return {
        "identical": (p1, p1.copy(), K),                      # no motion: every skew E fits
        "repeated": (np.repeat(p1[:8], 4, 0), np.repeat(p2[:8], 4, 0), K),  # 8 distinct pairs, 4 copies each
        "collinear": (line, line + [3.0, 0.0], K),            # all points on one line in both views
        "integer": (np.round(p1), np.round(p2), K),           # pixel-quantised, as ORB keypoints at level 0
        "pure_rotation": (p1, (p1 - [320, 240]) @ np.array([[0.99, -0.14], [0.14, 0.99]]) + [320, 240], K),
    }


@pytest.mark.parametrize("case", ["identical", "repeated", "collinear", "integer", "pure_rotation"])
def test_degenerate_correspondences(gpu_ctx, oracle_mod, case):
    """Degenerate point sets drive the 5-point solver into its rare branches
    (vanishing polynomial coefficients, coincident Durand-Kerner roots, rejected
    roots); the per-call findEssentialMat (one-round RANSAC, 16-lane Durand-Kerner
    and stage-C rows) must still agree with the oracle bit for bit."""
    from droplet_visual_odometry_amd import ops
    from droplet_visual_odometry_amd._native import DVOError
    p1, p2, K = _degenerate_sets()[case]
    p1 = np.ascontiguousarray(p1, dtype=np.float64)
    p2 = np.ascontiguousarray(p2, dtype=np.float64)
    Eo, mo, io = oracle_mod.find_essential(p1, p2, K)
    if Eo is None:
        with pytest.raises(DVOError):
            ops.find_essential_mat(p1, p2, K, ctx=gpu_ctx)
        return
    E, mask = ops.find_essential_mat(p1, p2, K, ctx=gpu_ctx)
    np.testing.assert_array_equal(E, Eo)
    np.testing.assert_array_equal(mask.ravel(), mo.ravel())


def test_detect_noise_frame_long_lists(gpu_ctx, oracle_mod):
    """A 1280x720 noise frame: ~90 K FAST survivors at level 0 (levels 0-4 past the
    per-call selection's LDS capacity of 8192, levels 5-7 inside it), so both the
    LDS and the global-memory retainBest paths run in one call, bit-exact."""
    from droplet_visual_odometry_amd import ops
    rng = np.random.default_rng(3)
    img = np.ascontiguousarray(rng.integers(0, 256, (720, 1280), dtype=np.uint8))
    kg, dg = ops.detect_and_compute(img, 2000, ctx=gpu_ctx)
    ko, do = oracle_mod.detect_and_compute(img, 2000)
    np.testing.assert_array_equal(kg.view(np.uint8), ko.view(np.uint8))
    np.testing.assert_array_equal(dg, do)


def test_large_batch_equals_small_batches(gpu_ctx):
    """An 800-frame batch (detection in two frame groups of 400, csrc/orb.hip launch_orb,
    DVO_ORB_GROUP 768) gives every frame the features and every pair the record that 2-frame
    batches of the same frames give, across the group boundary too (pair 399)."""
    import torch
    from droplet_visual_odometry_amd.stream import FrameStream
    W, H, N, F = 320, 240, 300, 800
    frames, K = synth_frames(W, H, range(F // 2))
    frames = np.concatenate([frames, frames])  # pair 399 closes the loop back to frame 0
    big = FrameStream(W, H, K, nfeatures=N, max_frames=F, ctx=gpu_ctx)
    dev = torch.from_numpy(np.ascontiguousarray(frames)).cuda()
    rec = big.process(dev)
    big.sync()
    recs = FrameStream.records_numpy(rec, F - 1)
    small = FrameStream(W, H, K, nfeatures=N, max_frames=2, ctx=gpu_ctx)
    for i in (0, 62, 398, 399, 400, 401, 767, 768, 798):
        r2 = small.process(dev[i:i + 2])
        small.sync()
        for k in (0, 1):
            kb, db = big.features(i + k)
            ks, ds = small.features(k)
            np.testing.assert_array_equal(kb.view(np.uint8), ks.view(np.uint8), err_msg=f"frame {i + k}")
            np.testing.assert_array_equal(db, ds, err_msg=f"frame {i + k}")
        rs = FrameStream.records_numpy(r2, 1)[0]
        for name in recs.dtype.names:
            if name not in ("pad0", "reserved"):
                np.testing.assert_array_equal(recs[i][name], rs[name], err_msg=f"pair {i} {name}")
    big.close()
    small.close()
    del dev
