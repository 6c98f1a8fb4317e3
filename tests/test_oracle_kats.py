"""CPU: pin the oracle (OpenCV restatement) with known-answer tests.

OpenCV itself is unavailable here, so the oracle is pinned by
(1) KAT-1, real OpenCV ORB output logged in the reference
(scripts/back_up_files/frame_extraction_notes.txt:6-7), (2) analytic inputs
with closed-form answers and (3) noise-free two-view geometry."""
import json
import math
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_kat1_keypoint_scale_arithmetic(oracle_mod):
    """Every logged ORB coordinate is float32(n) * the oracle's level scale
    float32(pow(double(1.2f), l)) (ora_orb_level_scales: nothing from the product package)."""
    scales = oracle_mod.level_scales(8)
    kat = json.load(open(os.path.join(HERE, "golden", "notes_kat1.json")))
    coords = [c for m in kat["matches"] for c in m["prev"] + m["cur"]]
    assert len(coords) == 40

    def explained(v, scale_fn):
        for l in range(8):
            s = scale_fn(l)
            n = round(v / float(s))
            if np.float32(np.float32(n) * s) == np.float32(v):
                return True
        return False

    ours = sum(explained(v, lambda l: scales[l]) for v in coords)
    naive = sum(explained(v, lambda l: np.float32(1.2 ** l)) for v in coords)
    assert ours == 40
    assert naive < 40  # the float32(1.2**l) hypothesis does not explain the log


def test_kat1_distances_are_hamming_integers():
    kat = json.load(open(os.path.join(HERE, "golden", "notes_kat1.json")))
    d = [m["distance"] for m in kat["matches"]]
    assert all(float(x).is_integer() and 0 <= x <= 256 for x in d)
    assert d == sorted(d)  # the reference's stable sort by distance (v3:221)


def test_oracle_keypoints_on_level_grid(oracle_mod, frames_640):
    frames, _ = frames_640
    kps, desc = oracle_mod.detect_and_compute(frames[0], 500)
    assert len(kps) == 500 and desc.shape == (500, 32)
    s = oracle_mod.level_scales(8)[kps["octave"]]
    xl = np.rint(kps["x"] / s)
    np.testing.assert_array_equal(np.float32(xl) * s, kps["x"])
    np.testing.assert_array_equal(kps["size"], np.float32(31) * s)
    assert np.all(np.diff(kps["octave"]) >= 0)  # level-major order
    assert np.all((kps["angle"] >= 0) & (kps["angle"] < 360))
    assert np.all(kps["class_id"] == -1)
    counts = np.bincount(kps["octave"], minlength=8)
    assert counts.tolist() == oracle_mod.features_per_level(500)


def test_pyramid_sizes_match_survey(oracle_mod):
    assert oracle_mod.level_sizes(1280, 720) == [(1280, 720), (1067, 600), (889, 500), (741, 417), (617, 347),
                                                 (514, 289), (429, 241), (357, 201)]
    assert oracle_mod.features_per_level(2000) == [434, 362, 302, 251, 209, 175, 145, 122]
    assert oracle_mod.features_per_level(500) == [109, 90, 75, 63, 52, 44, 36, 31]


def test_resize_and_blur_preserve_constant_image(oracle_mod):
    img = np.full((240, 320), 137, np.uint8)
    for lv in oracle_mod.pyramid(img):
        assert np.all(lv == 137)
    # the 8-bit Gaussian kernel sums to 257/256: a flat 137 blurs to (137*257*257 + 2^15) >> 16
    want = (137 * 257 * 257 + (1 << 15)) >> 16
    for lv in oracle_mod.pyramid(img, blurred=True):
        assert np.all(lv == want)


def test_gaussian_kernel_constants():
    g = np.exp(-np.arange(-3, 4) ** 2 / 8.0).astype(np.float32)
    k = np.rint(np.float64(g / g.sum()) * 256).astype(int)
    assert k.tolist() == [18, 34, 49, 55, 49, 34, 18]


def test_umax_table_matches_formula():
    half = 15
    vmax = math.floor(half * np.sqrt(np.float32(2)) / 2 + 1)
    vmin = math.ceil(half * np.sqrt(np.float32(2)) / 2)
    umax = [0] * (half + 2)
    for v in range(vmax + 1):
        umax[v] = int(np.rint(math.sqrt(half * half - v * v)))
    v0 = 0
    for v in range(half, vmin - 1, -1):
        while umax[v0] == umax[v0 + 1]:
            v0 += 1
        umax[v] = v0
        v0 += 1
    src = open(os.path.join(HERE, "..", "droplet_visual_odometry_amd", "csrc", "orb.hip")).read()
    assert "c_umax[16] = {" + ", ".join(map(str, umax[:16])) + "}" in src


def test_fast_analytic_corners(oracle_mod):
    """Isolated bright/dark pixels: each is a 16-of-16 FAST corner with score
    |v - background| - 1 (cornerScore<16>); a flat image has none; pixels
    within 3 of the border are never tested."""
    img = np.full((64, 64), 50, np.uint8)
    pos = [(10, 12, 200), (30, 40, 0), (50, 20, 71), (3, 30, 255), (20, 60, 255), (2, 10, 255), (61, 44, 255),
           (30, 2, 255), (40, 61, 0)]
    for x, y, v in pos:
        img[y, x] = v
    pts = oracle_mod.fast(img, 20)
    got = {(int(x), int(y)): int(s) for x, y, s in pts}
    # rows/cols 3 .. size-4 are tested (fast.cpp loops); score = |v - 50| - 1
    assert got == {(10, 12): 149, (30, 40): 49, (50, 20): 20, (3, 30): 204, (20, 60): 204}
    assert len(oracle_mod.fast(np.full((64, 64), 9, np.uint8), 20)) == 0


def test_retain_best_restated_introselect_matches_libstdcxx(oracle_mod):
    rng = np.random.default_rng(0)
    for n, k in [(4, 1), (5, 2), (17, 5), (100, 50), (1000, 217), (4000, 3999)]:
        for r in (rng.integers(0, 9, n).astype(np.float32), rng.standard_normal(n).astype(np.float32)):
            np.testing.assert_array_equal(oracle_mod.retain_best(r, k, depth=-1), oracle_mod.retain_best(r, k))
            kept = oracle_mod.retain_best(r, k)
            kth = np.sort(r)[::-1][k - 1]
            assert set(kept.tolist()) == set(np.nonzero(r >= kth)[0].tolist())


def test_retain_best_opencv32_semantics(oracle_mod):
    """OpenCV 3.2's retainBest (nth_element at n, boundary read at n - 1): the
    restated introselect equals libstdc++'s std::nth_element in this mode too;
    the kept set holds the n best, plus the tail entries tying the response now
    at index n - 1; and it differs from 4.x's when responses tie at the
    boundary (FAST scores are integers, so they usually do)."""
    rng = np.random.default_rng(1)
    differs = 0
    for n, k in [(4, 1), (5, 2), (17, 5), (100, 50), (1000, 217), (4000, 3999)]:
        for r in (rng.integers(0, 9, n).astype(np.float32), rng.standard_normal(n).astype(np.float32)):
            kept = oracle_mod.retain_best(r, k, semantics=oracle_mod.OCV32)
            np.testing.assert_array_equal(oracle_mod.retain_best(r, k, depth=-1, semantics=oracle_mod.OCV32), kept)
            assert len(kept) >= k
            kth = np.sort(r)[::-1][k - 1]
            assert set(np.nonzero(r > kth)[0].tolist()) <= set(kept.tolist()) <= set(np.nonzero(r >= kth)[0].tolist())
            differs += set(kept.tolist()) != set(oracle_mod.retain_best(r, k).tolist())
    assert differs > 0


def test_opencv32_pyramid_kats(oracle_mod):
    """resize(INTER_LINEAR) as 3.2 ran it: a constant image stays constant
    wherever both 11-bit weights round to a 2048 sum, the SSE2 / scalar split
    sits where its loops stop, and the 3.2 pyramid differs from 4.x's
    INTER_LINEAR_EXACT one on a textured frame (level 0 is the input in both)."""
    from conftest import synth_frames
    frames, _ = synth_frames(640, 480, [0])
    a = oracle_mod.pyramid(frames[0], semantics=oracle_mod.OCV4)
    b = oracle_mod.pyramid(frames[0], semantics=oracle_mod.OCV32)
    np.testing.assert_array_equal(a[0], b[0])
    assert all(x.shape == y.shape for x, y in zip(a, b))
    assert any(not np.array_equal(x, y) for x, y in zip(a[1:], b[1:]))
    # the SSE2 vertical pass truncates twice (h >> 4, mulhi): each 3.2 level comes out about
    # 0.12 grey levels darker than the bit-exact one, and levels are resized from levels
    for l in range(1, 8):
        d = b[l].astype(int) - a[l].astype(int)
        assert -0.15 * l < float(d.mean()) < -0.09 * l and np.abs(d).max() <= 3
    for v in (0, 1, 128, 255):
        lv = oracle_mod.pyramid(np.full((96, 128), v, np.uint8), semantics=oracle_mod.OCV32)
        for L in lv:
            assert abs(int(L.min()) - v) <= 1 and abs(int(L.max()) - v) <= 1


def test_blur_rounds_ties_half_even_except_last_columns(oracle_mod):
    """GaussianBlur's column pass (SymmColumnVec_32s8u) rounds sum / 2^16 half to
    even in float; only the last w % 4 columns take the scalar (sum + 2^15) >> 16.
    Checked against exact integer sums on a frame with ties."""
    from conftest import synth_frames
    frames, _ = synth_frames(640, 480, [1])
    k = np.array([18, 34, 49, 55, 49, 34, 18])

    def refl(n):
        i = np.arange(-3, n + 3)
        i = np.where(i < 0, -i, i)
        return np.where(i >= n, 2 * n - 2 - i, i)
    ties = 0
    for L, B in zip(oracle_mod.pyramid(frames[0]), oracle_mod.pyramid(frames[0], blurred=True)):
        h, w = L.shape
        a = L.astype(np.int64)[:, refl(w)]
        rows = sum(k[i] * a[:, i:i + w] for i in range(7))[refl(h), :]
        S = sum(k[i] * rows[i:i + h, :] for i in range(7))
        want = np.minimum((S + 32768) >> 16, 255)
        he = np.minimum((S + 32767 + ((S >> 16) & 1)) >> 16, 255)
        want[:, :w & ~3] = he[:, :w & ~3]
        np.testing.assert_array_equal(B, want)
        ties += int(((S & 0xFFFF) == 0x8000).sum())
    assert ties > 0


def test_bf_match_tie_rules(oracle_mod):
    d = np.zeros((4, 32), np.uint8)
    d[1, 0] = 1      # distance 1 from d[0]
    d[2, 0] = 3      # distance 2
    d[3] = 255       # far
    t = np.zeros((3, 32), np.uint8)
    t[1] = d[3]
    t[2] = d[1]
    q, tt, dist = oracle_mod.bf_match(d, t, 1)
    # query 0 -> train 0 (d 0, first of ties); query 1 -> train 2 (d 0); query 3 -> train 1
    assert list(zip(q, tt, dist)) == [(0, 0, 0.0), (1, 2, 0.0), (3, 1, 0.0)]
    q0, t0, _ = oracle_mod.bf_match(d, t, 0)
    assert list(q0) == [0, 1, 2, 3] and t0[2] == 2  # no cross check: q2 keeps its forward NN


def _two_view(rng, n=80, noise=0.0):
    K = np.array([[600.0, 0, 320], [0, 610.0, 240], [0, 0, 1]])
    ang = 0.07
    ax = np.array([0.2, 1.0, 0.1])
    ax /= np.linalg.norm(ax)
    Kx = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    R = np.eye(3) + math.sin(ang) * Kx + (1 - math.cos(ang)) * Kx @ Kx
    t = np.array([0.4, -0.1, 0.9])
    t /= np.linalg.norm(t)
    X = np.c_[rng.uniform(-3, 3, n), rng.uniform(-2.5, 2.5, n), rng.uniform(2, 6, n)]
    x1 = X @ K.T
    x1 = x1[:, :2] / x1[:, 2:]
    X2 = X @ R.T + 1.0 * t
    x2 = X2 @ K.T
    x2 = x2[:, :2] / x2[:, 2:]
    return K, R, t, X, x1 + rng.normal(0, noise, x1.shape), x2 + rng.normal(0, noise, x2.shape)


def test_geometry_noise_free_recovers_truth(oracle_mod):
    rng = np.random.default_rng(3)
    K, R, t, X, x1, x2 = _two_view(rng)
    E, mask, iters = oracle_mod.find_essential(x1, x2, K)
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
    Et = tx @ R
    Et /= np.linalg.norm(Et)
    assert min(np.abs(E - Et).max(), np.abs(E + Et).max()) < 1e-9
    assert mask.sum() == len(x1) and iters == 1
    good, Rr, tr, pm = oracle_mod.recover_pose(E, x1, x2, K)
    assert good == len(x1)
    assert np.abs(Rr - R).max() < 1e-9 and np.abs(tr.ravel() - t).max() < 1e-9
    P1 = K @ np.c_[np.eye(3), np.zeros(3)]
    P2 = K @ np.c_[R, 1.0 * t]
    Xh = oracle_mod.triangulate(P1, P2, x1.T.copy(), x2.T.copy())
    np.testing.assert_allclose((Xh[:3] / Xh[3]).T, X, rtol=1e-9, atol=1e-9)


def test_five_point_contains_true_essential(oracle_mod):
    rng = np.random.default_rng(11)
    K, R, t, X, x1, x2 = _two_view(rng, n=5)
    n1 = (x1 - K[:2, 2]) / [K[0, 0], K[1, 1]]
    n2 = (x2 - K[:2, 2]) / [K[0, 0], K[1, 1]]
    Ms = oracle_mod.five_point(n1, n2)
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
    Et = tx @ R
    Et /= np.linalg.norm(Et)
    assert 1 <= len(Ms) <= 10
    assert min(min(np.abs(M - Et).max(), np.abs(M + Et).max()) for M in Ms) < 1e-8
    for M in Ms:  # every model satisfies the 5 epipolar constraints
        h1 = np.c_[n1, np.ones(5)]
        h2 = np.c_[n2, np.ones(5)]
        assert np.abs(np.einsum("ij,jk,ik->i", h2, M, h1)).max() < 1e-9


def test_jacobi_svd_matches_numpy(oracle_mod):
    rng = np.random.default_rng(1)
    for shape in [(3, 3), (4, 4), (9, 5), (6, 2)]:
        A = rng.standard_normal(shape)
        W, U, Vt = oracle_mod.jacobi_svd(A, full_u=True)
        np.testing.assert_allclose(W, np.linalg.svd(A, compute_uv=False), rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(U[:, :len(W)] * W @ Vt, A, atol=1e-12)
        assert np.all(np.diff(W) <= 0)


def test_solve_poly_roots(oracle_mod):
    c = np.polynomial.polynomial.polyfromroots(np.arange(1, 11, dtype=float))
    roots = oracle_mod.solve_poly(c)
    assert len(roots) == 10
    np.testing.assert_allclose(np.sort(roots[:, 0]), np.arange(1, 11), atol=1e-6)
    assert np.abs(roots[:, 1]).max() < 1e-8


def test_ransac_update_num_iters_formula(oracle_mod):
    f = oracle_mod.ransac_update_num_iters
    assert f(0.999, 0.0, 5, 1000) == 0                    # all inliers: stop
    assert f(0.999, 1.0, 5, 1000) == 1000                 # no inliers: keep max
    want = int(np.rint(math.log(0.001) / math.log(1 - 0.5 ** 5)))
    assert f(0.999, 0.5, 5, 1000) == want == 218
    assert f(0.999, 0.9, 5, 1000) == 1000


def test_rng_multiply_with_carry():
    """cv::RNG(uint64(-1)): state = (u32)state * 4164903690 + (state >> 32)."""
    s = (1 << 64) - 1
    out = []
    for _ in range(3):
        s = (s & 0xFFFFFFFF) * 4164903690 + (s >> 32)
        out.append(s & 0xFFFFFFFF)
    assert out[0] == (0xFFFFFFFF * 4164903690 + 0xFFFFFFFF) & 0xFFFFFFFF
    assert len(set(out)) == 3


def test_golden_pair_reproduces(oracle_mod):
    g = np.load(os.path.join(HERE, "golden", "pair_320x240.npz"))
    f = g["frames"]
    kp0, d0 = oracle_mod.detect_and_compute(f[0], int(g["nfeatures"]))
    np.testing.assert_array_equal(kp0.view(np.uint8), g["kp0"].view(np.uint8))
    np.testing.assert_array_equal(d0, g["desc0"])
    r = oracle_mod.pair_pose(f[0], f[1], g["K"], int(g["nfeatures"]), kp_prev=(kp0, d0))
    np.testing.assert_array_equal(r["q"], g["q"])
    np.testing.assert_array_equal(r["t"], g["t"])
    np.testing.assert_array_equal(r["E"], g["E"])
    np.testing.assert_array_equal(r["R"], g["R"])
    np.testing.assert_array_equal(r["t_unit"], g["t_unit"])
    assert r["good"] == int(g["good"]) and r["iters"] == int(g["iters"])


def test_oracle_subsets_follow_cv_rng(oracle_mod):
    """getSubset's draws from cv::RNG((uint64)-1): state = (uint32)state *
    4164903690 + (state >> 32), uniform(0, m) = (uint32)state % m, a draw
    repeating an earlier index of the subset is redrawn."""
    def ref(m, n):
        st, out = (1 << 64) - 1, []
        for _ in range(n):
            v = []
            for _ in range(5):
                while True:
                    st = ((st & 0xFFFFFFFF) * 4164903690 + (st >> 32)) & ((1 << 64) - 1)
                    x = (st & 0xFFFFFFFF) % m
                    if x not in v:
                        break
                v.append(x)
            out.append(v)
        return out
    for m, n in [(6, 50), (9, 200), (871, 300)]:
        assert oracle_mod.ransac_subsets(m, n).tolist() == ref(m, n)


def test_surf_restatement_invariants(oracle_mod):
    """oracle/surf.cpp (SURF_create(400), the 'surf' mode, v3:104): keypoints in
    KeypointGreater order, sizes integral after interpolation, class_id the
    sign of the Hessian trace, unit-norm 64-d descriptors, orientation in
    [0, 360), octaves 0..3.  (OpenCV's own output is not available here:
    parity against it is unpinned.)"""
    from conftest import synth_frames
    frames, _ = synth_frames(320, 240, range(1))
    k, d = oracle_mod.surf_detect_and_compute(frames[0], 400.0)
    assert len(k) > 100 and d.shape == (len(k), 64)
    np.testing.assert_allclose(np.linalg.norm(d, axis=1), 1.0, rtol=1e-5)
    assert np.all(np.diff(k["response"]) <= 0)
    assert np.all(k["size"] == np.round(k["size"])) and np.all(k["size"] >= 9 - 6)
    assert set(np.unique(k["class_id"])) <= {-1, 1}
    assert np.all((k["angle"] >= 0) & (k["angle"] < 360))
    assert set(np.unique(k["octave"])) <= {0, 1, 2, 3}
    k2, d2 = oracle_mod.surf_detect_and_compute(frames[0], 800.0)
    assert len(k2) < len(k) and np.all(k2["response"] > 800)


def test_product_level_scale_equals_oracle(oracle_mod):
    """The product's host plan places keypoints with the oracle's level scales, bit for bit."""
    from droplet_visual_odometry_amd.plan import level_scale
    got = np.array([level_scale(l) for l in range(8)], np.float32)
    assert got.tobytes() == oracle_mod.level_scales(8).tobytes()
