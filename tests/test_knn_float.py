"""Float-descriptor matching (the SIFT / SURF / knn_sift /
flann modes, visual_odometry_v3.py:99-106, :200-228).

CPU: the oracle's BFMatcher(NORM_L1).knnMatch / FLANN squared-L2 restatement
(oracle/match.cpp ora_bf_knn_float) against an independent numpy brute force
on SIFT-like integer-valued descriptors, where every summation order gives the
same float (so the check is order-free), including OpenCV's tie rule (lower
train index first) and padding; cv shim host logic.  GPU: the HIP kernel
through the C-ABI, bit-exact against the oracle on integer-valued and on
arbitrary float descriptors, chunk-crossing ties, tiny and ragged sizes, the
cv shim and the drop-in's ratio-test modes.  Parity vs OpenCV itself is
unpinned (cv2 is absent; its SIMD L1 sums in another order, which matters only
for non-integer descriptors such as SURF's)."""
import numpy as np
import pytest

FLT_MAX = np.finfo(np.float32).max


def sift_like(rng, n, dim=128):
    return rng.integers(0, 256, (n, dim)).astype(np.float32)


def brute(dq, dt, k, norm):
    a = dq.astype(np.int64)[:, None, :] - dt.astype(np.int64)[None, :, :]
    d = np.abs(a).sum(-1) if norm == 0 else (a * a).sum(-1)
    nq, nt = d.shape
    idx = np.full((nq, k), -1, np.int32)
    dist = np.full((nq, k), FLT_MAX, np.float32)
    for q in range(nq):
        order = np.lexsort((np.arange(nt), d[q]))[:k]
        idx[q, :len(order)] = order
        dist[q, :len(order)] = d[q, order]
    return idx, dist


@pytest.mark.parametrize("norm", [0, 1])
@pytest.mark.parametrize("k", [1, 2, 3])
def test_oracle_matches_bruteforce_integer_descriptors(oracle_mod, norm, k):
    rng = np.random.default_rng(10 * norm + k)
    dq = sift_like(rng, 37)
    dt = sift_like(rng, 53)
    dt[20] = dt[3]      # duplicate trains -> equal distances, lower index first
    dt[41] = dt[3]
    dq[5] = dt[3]
    i_o, d_o = oracle_mod.bf_knn_float(dq, dt, k, norm)
    i_b, d_b = brute(dq, dt, k, norm)
    np.testing.assert_array_equal(i_o, i_b)
    np.testing.assert_array_equal(d_o, d_b)
    if k >= 3:
        assert list(i_o[5, :3]) == [3, 20, 41] and d_o[5, 0] == 0


def test_oracle_pads_when_fewer_trains_than_k(oracle_mod):
    rng = np.random.default_rng(3)
    i_o, d_o = oracle_mod.bf_knn_float(sift_like(rng, 4, 64), sift_like(rng, 1, 64), 2, 0)
    assert (i_o[:, 0] == 0).all() and (i_o[:, 1] == -1).all() and (d_o[:, 1] == FLT_MAX).all()


def test_cv_shim_host_checks():
    from droplet_visual_odometry_amd import cv
    bf = cv.BFMatcher(cv.NORM_L1, crossCheck=False)
    q = np.zeros((3, 128), np.float32)
    assert bf.knnMatch(q, np.zeros((0, 128), np.float32), k=2) == [[], [], []]
    assert bf.knnMatch(np.zeros((0, 128), np.float32), q, k=2) == []
    with pytest.raises(cv.error):
        bf.knnMatch(q.astype(np.uint8), q, k=2)
    with pytest.raises(cv.error):
        cv.BFMatcher(cv.NORM_L1, crossCheck=True).knnMatch(q, q, k=2)
    with pytest.raises(cv.error):
        cv.BFMatcher(cv.NORM_L2).match(q, q)


# ---------------------------------------------------------------------------- GPU


@pytest.mark.gpu
@pytest.mark.parametrize("dim", [128, 64])
@pytest.mark.parametrize("norm", [0, 1])
@pytest.mark.parametrize("k", [1, 2, 4])
def test_gpu_knn_bit_exact_integer_descriptors(gpu_ctx, oracle_mod, dim, norm, k):
    from droplet_visual_odometry_amd import ops
    rng = np.random.default_rng(dim + 7 * norm + k)
    dq = sift_like(rng, 1500, dim)
    dt = sift_like(rng, 1301, dim)
    for a, b in [(5, 69), (5, 700), (5, 1300), (64, 65)]:   # ties across train chunks of 64
        dt[b] = dt[a]
    dq[:40] = dt[5]
    i_g, d_g = ops.bf_knn_float(dq, dt, k, norm, ctx=gpu_ctx)
    i_o, d_o = oracle_mod.bf_knn_float(dq, dt, k, norm)
    np.testing.assert_array_equal(i_g, i_o)
    np.testing.assert_array_equal(d_g.view(np.uint32), d_o.view(np.uint32))
    if k >= 2:
        assert (i_g[:40, 0] == 5).all() and (i_g[:40, 1] == 69).all()


@pytest.mark.gpu
@pytest.mark.parametrize("norm", [0, 1])
def test_gpu_knn_bit_exact_real_valued(gpu_ctx, oracle_mod, norm):
    """Non-integer (SURF-like, unit-norm 64-d) descriptors: the kernel sums in
    the restated order without contraction, so it is bit-exact to the oracle."""
    from droplet_visual_odometry_amd import ops
    rng = np.random.default_rng(100 + norm)
    dq = rng.standard_normal((777, 64)).astype(np.float32)
    dt = rng.standard_normal((901, 64)).astype(np.float32)
    dq /= np.linalg.norm(dq, axis=1, keepdims=True)
    dt /= np.linalg.norm(dt, axis=1, keepdims=True)
    i_g, d_g = ops.bf_knn_float(dq, dt, 2, norm, ctx=gpu_ctx)
    i_o, d_o = oracle_mod.bf_knn_float(dq, dt, 2, norm)
    np.testing.assert_array_equal(i_g, i_o)
    np.testing.assert_array_equal(d_g.view(np.uint32), d_o.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("nq,nt", [(1, 1), (1, 2), (3, 1), (257, 63), (256, 64), (255, 65), (5000, 4000),
                                   (20000, 1500)])
def test_gpu_knn_sizes(gpu_ctx, oracle_mod, nq, nt):
    from droplet_visual_odometry_amd import ops
    rng = np.random.default_rng(nq * 7 + nt)
    dq, dt = sift_like(rng, nq), sift_like(rng, nt)
    i_g, d_g = ops.bf_knn_float(dq, dt, 2, 0, ctx=gpu_ctx)
    i_o, d_o = oracle_mod.bf_knn_float(dq, dt, 2, 0)
    np.testing.assert_array_equal(i_g, i_o)
    np.testing.assert_array_equal(d_g, d_o)


@pytest.mark.gpu
def test_gpu_knn_rejects_bad_arguments(gpu_ctx):
    from droplet_visual_odometry_amd import ops
    from droplet_visual_odometry_amd._native import DVOError
    q = np.zeros((4, 96), np.float32)
    with pytest.raises(DVOError):
        ops.bf_knn_float(q, q, 2, 0, ctx=gpu_ctx)          # dim 96
    q = np.zeros((4, 128), np.float32)
    with pytest.raises(DVOError):
        ops.bf_knn_float(q, q, 5, 0, ctx=gpu_ctx)          # k 5
    with pytest.raises(DVOError):
        ops.bf_knn_float(q, q, 2, 3, ctx=gpu_ctx)          # norm


@pytest.mark.gpu
def test_cv_matchers_and_ratio_modes(gpu_ctx, oracle_mod):
    """BFMatcher(NORM_L1).match/knnMatch, FlannBasedMatcher.knnMatch and the
    drop-in's ratio test (v3:223-228) against the oracle."""
    from droplet_visual_odometry_amd import cv
    rng = np.random.default_rng(42)
    prev = sift_like(rng, 600)
    cur = np.concatenate([prev[:400] + rng.integers(-3, 4, (400, 128)), sift_like(rng, 300)]).astype(np.float32)
    cur = np.clip(cur, 0, 255)
    bf = cv.BFMatcher(normType=cv.NORM_L1, crossCheck=False)
    i_o, d_o = oracle_mod.bf_knn_float(prev, cur, 2, 0)
    knn = bf.knnMatch(prev, cur, k=2)
    assert len(knn) == 600 and all(len(r) == 2 for r in knn)
    assert [(r[0].trainIdx, r[1].trainIdx) for r in knn] == [tuple(x) for x in i_o]
    assert [r[0].distance for r in knn] == [float(x) for x in d_o[:, 0]]
    single = bf.match(prev, cur)
    assert [(m.queryIdx, m.trainIdx, m.distance) for m in single] == \
        [(q, int(i_o[q, 0]), float(d_o[q, 0])) for q in range(600)]
    passed = [[m] for m, n in knn if m.distance < 0.75 * n.distance]
    expect = [q for q in range(600) if float(d_o[q, 0]) < 0.75 * float(d_o[q, 1])]
    assert [p[0].queryIdx for p in passed] == expect and len(expect) >= 350
    cv.setRNGSeed(0)  # a fresh thread's cv::theRNG()
    i_f, d_f, _ = oracle_mod.flann_knn(prev, cur, 2, trees=5, checks=50)
    fl = cv.FlannBasedMatcher(dict(algorithm=1, trees=5), dict(checks=50)).knnMatch(prev, cur, k=2)
    # DMatch.distance = std::sqrt(float squared-L2), FlannBasedMatcher::convertToDMatches
    s_f = np.sqrt(d_f.astype(np.float32))
    assert [(r[0].trainIdx, r[1].trainIdx, r[0].distance, r[1].distance) for r in fl] == \
        [(int(a), int(b), float(c), float(d)) for (a, b), (c, d) in zip(i_f, s_f)]
    fl_pass = [q for q, (m, n) in enumerate(fl) if m.distance < 0.75 * n.distance]
    assert fl_pass == [q for q in range(600) if float(s_f[q, 0]) < 0.75 * float(s_f[q, 1])]
    # the ratio on squared distances would be an effective 0.866 and can only pass more
    assert len(fl_pass) <= sum(float(d_f[q, 0]) < 0.75 * float(d_f[q, 1]) for q in range(600))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["knn_sift", "surf", "flann"])
def test_dropin_ratio_modes(gpu_ctx, oracle_mod, mode):
    """VisualOdometry.get_matches_between_two_frames (v3:191-239) in the
    k-NN modes: the keypoints that pass the 0.75 ratio test, in query order."""
    import os
    import sys
    import types
    from droplet_visual_odometry_amd import cv
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "droplet_visual_odometry_amd", "dropin"))
    try:
        import visual_odometry_v3 as v3
    finally:
        sys.path.pop(0)
    rng = np.random.default_rng(7)
    dim = 64 if mode == "surf" else 128
    prev = sift_like(rng, 300, dim)
    cur = np.clip(np.concatenate([prev[:200] + rng.integers(-2, 3, (200, dim)), sift_like(rng, 150, dim)]),
                  0, 255).astype(np.float32)
    kp_prev = [cv.KeyPoint(float(i), 0.0) for i in range(300)]
    kp_cur = [cv.KeyPoint(float(i), 1.0) for i in range(350)]
    me = types.SimpleNamespace(mode=mode, bf=cv.BFMatcher(normType=cv.NORM_L1, crossCheck=False))
    cv.setRNGSeed(0)
    matches, top_prev, top_cur = v3.VisualOdometry.get_matches_between_two_frames(me, kp_prev, prev, kp_cur, cur)
    if mode == "flann":  # FLANN's DMatch.distance is sqrt(float) of the squared L2 distance
        idx, dist, _ = oracle_mod.flann_knn(prev, cur, 2, trees=5, checks=50)
        dist = np.sqrt(dist.astype(np.float32))
    else:
        idx, dist = oracle_mod.bf_knn_float(prev, cur, 2, 0)
    keep = [q for q in range(300) if float(dist[q, 0]) < 0.75 * float(dist[q, 1])]
    assert len(matches) == 300 and len(keep) >= 150
    assert [kp.pt[0] for kp in top_prev] == [float(q) for q in keep]
    assert [kp.pt[0] for kp in top_cur] == [float(idx[q, 0]) for q in keep]


@pytest.mark.gpu
def test_dropin_sift_mode_fails_in_ratio_loop_like_the_reference(gpu_ctx):
    """'sift' mode calls bf.match (v3:200-201) and then unpacks `for m, n in
    matches` (v3:226): single DMatch objects do not unpack into two, so the
    reference raises there (cv2: TypeError); the drop-in raises too."""
    import os
    import sys
    import types
    from droplet_visual_odometry_amd import cv
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "droplet_visual_odometry_amd", "dropin"))
    try:
        import visual_odometry_v3 as v3
    finally:
        sys.path.pop(0)
    rng = np.random.default_rng(1)
    d = sift_like(rng, 20)
    kps = [cv.KeyPoint(float(i), 0.0) for i in range(20)]
    me = types.SimpleNamespace(mode="sift", bf=cv.BFMatcher(normType=cv.NORM_L1, crossCheck=False))
    with pytest.raises((TypeError, ValueError)):
        v3.VisualOdometry.get_matches_between_two_frames(me, kps, d, kps, d)


@pytest.mark.gpu
@pytest.mark.parametrize("poison", [255.5, 300.0, -1.0, 0.25])
@pytest.mark.parametrize("norm", [0, 1])
def test_gpu_knn_non_byte_values_take_the_float_path(gpu_ctx, oracle_mod, poison, norm):
    """One value outside the byte fast path (non-integer, > 255 or negative,
    in queries or trains) sends the whole call to the float kernel: results
    stay bit-exact to the oracle either way."""
    from droplet_visual_odometry_amd import ops
    rng = np.random.default_rng(int(abs(poison) * 4) + norm)
    dq, dt = sift_like(rng, 700), sift_like(rng, 900)
    for a, who in [(dq, "q"), (dt, "t")]:
        b = a.copy()
        b[17, 33] = poison
        q, t = (b, dt) if who == "q" else (dq, b)
        i_g, d_g = ops.bf_knn_float(q, t, 2, norm, ctx=gpu_ctx)
        i_o, d_o = oracle_mod.bf_knn_float(q, t, 2, norm)
        np.testing.assert_array_equal(i_g, i_o)
        np.testing.assert_array_equal(d_g.view(np.uint32), d_o.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("norm", [0, 1])
def test_gpu_knn_byte_path_extremes(gpu_ctx, oracle_mod, norm):
    """Byte path at its range limits: all-0 against all-255 rows give the
    largest distances (L2^2 = 128 * 255^2 = 8,323,200 < 2^24, still exact),
    and -0.0 counts as the byte 0; ties across the 64-row LDS stages keep
    the lower train index."""
    from droplet_visual_odometry_amd import ops
    rng = np.random.default_rng(7 + norm)
    dq, dt = sift_like(rng, 300), sift_like(rng, 700)
    dq[:10] = 0.0
    dq[10:20] = 255.0
    dq[20:30] = -0.0
    dt[::2] = 255.0  # many equal far rows; ties straddle LDS stages
    dt[1::50] = 0.0
    for k in (1, 2, 4):
        i_g, d_g = ops.bf_knn_float(dq, dt, k, norm, ctx=gpu_ctx)
        i_o, d_o = oracle_mod.bf_knn_float(dq, dt, k, norm)
        np.testing.assert_array_equal(i_g, i_o)
        np.testing.assert_array_equal(d_g.view(np.uint32), d_o.view(np.uint32))
