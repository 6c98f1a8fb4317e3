"""GPU vs oracle parity through the C ABI (bit-exact for keypoints, descriptors,
matches and RANSAC hypotheses; E / R / t bit-identical by construction, checked
at 0 ulp with a 1e-12 fallback bound printed on failure)."""
import numpy as np
import pytest

from conftest import synth_frames

pytestmark = pytest.mark.gpu


def test_library_loaded_from_repo(gpu_ctx):
    import droplet_visual_odometry_amd._native as N
    assert N._lib is not None and N._lib._name == N.LIB_PATH
    assert N._lib.dvo_version() == 1


def test_detect_and_compute_640(gpu_ctx, oracle_mod, frames_640):
    from droplet_visual_odometry_amd import ops
    frames, _ = frames_640
    for f in frames[:2]:
        kg, dg = ops.detect_and_compute(f, 500, ctx=gpu_ctx)
        ko, do = oracle_mod.detect_and_compute(f, 500)
        assert len(kg) == len(ko)
        np.testing.assert_array_equal(kg.view(np.uint8), ko.view(np.uint8))
        np.testing.assert_array_equal(dg, do)


@pytest.mark.parametrize("n,npoints", [(10, 3), (1000, 217), (5000, 434), (20000, 868), (333, 333), (7, 0)])
def test_retain_best_matches_libstdcxx(gpu_ctx, oracle_mod, n, npoints):
    from droplet_visual_odometry_amd import ops
    rng = np.random.default_rng(n)
    for trial in range(3):
        if trial == 0:
            r = rng.integers(21, 60, n).astype(np.float32)        # FAST-like ties
        elif trial == 1:
            r = rng.standard_normal(n).astype(np.float32)
        else:
            r = np.full(n, 5.0, np.float32)
        want = oracle_mod.retain_best(r, npoints)
        got = ops.test_retain_best(r, npoints, ctx=gpu_ctx)
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("depth", [0, 1, 2, 3])
def test_retain_best_heap_select_path(gpu_ctx, oracle_mod, depth):
    from droplet_visual_odometry_amd import ops
    rng = np.random.default_rng(depth)
    r = rng.integers(0, 40, 3000).astype(np.float32)
    want = oracle_mod.retain_best(r, 300, depth=depth)
    got = ops.test_retain_best(r, 300, depth=depth, ctx=gpu_ctx)
    np.testing.assert_array_equal(got, want)
    # the restated introselect equals libstdc++'s at the default depth
    np.testing.assert_array_equal(oracle_mod.retain_best(r, 300, depth=-1), oracle_mod.retain_best(r, 300))


def test_update_num_iters(gpu_ctx, oracle_mod):
    from droplet_visual_odometry_amd import ops
    m = np.arange(5, 2100)
    eps = np.concatenate([(m - g) / m for g in (5, 6, 37)] + [np.linspace(0, 1, 5001)])
    got = ops.test_update_num_iters(0.999, eps, 5, 1000, ctx=gpu_ctx)
    want = np.array([oracle_mod.ransac_update_num_iters(0.999, e, 5, 1000) for e in eps])
    np.testing.assert_array_equal(got, want)


def test_five_point(gpu_ctx, oracle_mod):
    from droplet_visual_odometry_amd import ops
    rng = np.random.default_rng(5)
    for _ in range(20):
        q1 = rng.uniform(-0.6, 0.6, (5, 2))
        q2 = q1 + rng.normal(0, 0.05, (5, 2))
        want = oracle_mod.five_point(q1, q2)
        got = ops.test_five_point(q1, q2, ctx=gpu_ctx)
        assert got.shape == want.shape
        np.testing.assert_array_equal(got, want)


def test_bf_match(gpu_ctx, oracle_mod, frames_640):
    from droplet_visual_odometry_amd import ops
    frames, _ = frames_640
    _, d0 = oracle_mod.detect_and_compute(frames[0], 500)
    _, d1 = oracle_mod.detect_and_compute(frames[1], 500)
    for mode in (0, 1, 2):
        q, t, d = oracle_mod.bf_match(d0, d1, mode)
        got = ops.bf_match(d0, d1, mode, ctx=gpu_ctx)
        np.testing.assert_array_equal(got["queryIdx"], q)
        np.testing.assert_array_equal(got["trainIdx"], t)
        np.testing.assert_array_equal(got["distance"], d)


def test_essential_and_pose(gpu_ctx, oracle_mod, frames_640):
    from droplet_visual_odometry_amd import ops
    frames, K = frames_640
    for i in range(2):
        ref = oracle_mod.pair_pose(frames[i], frames[i + 1], K, 500)
        E, mask = ops.find_essential_mat(ref["p1"], ref["p2"], K, ctx=gpu_ctx)
        np.testing.assert_array_equal(E, ref["E"])
        good, R, t, pm = ops.recover_pose(E, ref["p1"], ref["p2"], K, ctx=gpu_ctx)
        assert good == ref["good"]
        np.testing.assert_array_equal(R, ref["R"])
        np.testing.assert_array_equal(t, ref["t_unit"])


def test_stream_end_to_end_640(gpu_ctx, oracle_mod, frames_640):
    import torch
    from droplet_visual_odometry_amd.stream import FrameStream
    frames, K = frames_640
    fs = FrameStream(640, 480, K, nfeatures=500, max_frames=8, ctx=gpu_ctx)
    dev = torch.from_numpy(frames).cuda()
    rec = fs.process(dev)
    fs.sync()
    recs = FrameStream.records_numpy(rec, len(frames) - 1)
    kp_prev = None
    for i in range(len(frames) - 1):
        ref = oracle_mod.pair_pose(frames[i], frames[i + 1], K, 500, kp_prev=kp_prev)
        kp_prev = (ref["kp_cur"], ref["desc_cur"])
        kg, dg = fs.features(i + 1)
        np.testing.assert_array_equal(kg.view(np.uint8), ref["kp_cur"].view(np.uint8))
        mg = fs.matches(i)
        np.testing.assert_array_equal(mg["queryIdx"], ref["q"])
        np.testing.assert_array_equal(mg["trainIdx"], ref["t"])
        r = recs[i]
        assert r["status"] == 0
        assert r["n_matches"] == len(ref["q"])
        assert r["ransac_iters"] == ref["iters"]
        np.testing.assert_array_equal(r["E"].reshape(3, 3), ref["E"])
        np.testing.assert_array_equal(r["R"].reshape(3, 3), ref["R"])
        np.testing.assert_array_equal(r["t"], ref["t_unit"].ravel())
        assert r["n_good"] == ref["good"]


@pytest.mark.parametrize("nq,nt", [(1, 1), (5, 300), (63, 64), (257, 255), (2000, 2000), (4000, 3500), (700, 8192),
                                   (8192, 8192)])
def test_bf_match_sizes(gpu_ctx, oracle_mod, nq, nt):
    """Per-call BFMatcher(NORM_HAMMING).match (v3:219) on the MFMA matcher at
    ragged sizes up to the 8192 cap, every crossCheck mode, bit-exact.  Half the
    descriptors are low-entropy (few set bits), so distance ties across the
    train split and the LDS stages are common."""
    from droplet_visual_odometry_amd import ops
    rng = np.random.default_rng(nq * 7 + nt)
    dq = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    dt = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
    dq[::2] &= rng.integers(0, 256, (len(dq[::2]), 32), dtype=np.uint8) & 0x11
    dt[::2] &= rng.integers(0, 256, (len(dt[::2]), 32), dtype=np.uint8) & 0x11
    if nt > 4:
        dt[nt // 2] = dt[1]  # an exact duplicate train: the lower index must win
    for mode in (0, 1, 2):
        q, t, d = oracle_mod.bf_match(dq, dt, mode)
        got = ops.bf_match(dq, dt, mode, ctx=gpu_ctx)
        np.testing.assert_array_equal(got["queryIdx"], q)
        np.testing.assert_array_equal(got["trainIdx"], t)
        np.testing.assert_array_equal(got["distance"], d)
