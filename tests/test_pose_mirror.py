"""recoverPose's [R|t] / [R|-t] mirror (csrc/geometry.hip pose_count_kernel),
checked on the host with the oracle's own triangulatePoints (oracle/geometry.cpp, the same
Jacobi SVD restatement the device compiles): triangulating against [R|-t] gives exactly
sigma (X0, X1, X2, -X3) of the [R|t] result (sigma = +-1; IEEE rounding is symmetric, so the
Jacobi sweeps stay exact negations of each other), and the cheirality / distance tests of the
-t decomposition computed from the +t point with negated X2 X3, q and z equal the tests on
its own triangulation (five_point.cpp recoverPose, visual_odometry_v3.py:303)."""
import numpy as np


def _rot(rng):
    q = rng.standard_normal(4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def _tests(X, P, d, mirror):
    with np.errstate(all="ignore"):
        if not mirror:
            ok = X[2] * X[3] > 0
            q = X / X[3]
            ok &= q[2] < d
            z = P[2, 0] * q[0] + P[2, 1] * q[1] + P[2, 2] * q[2] + P[2, 3] * q[3]
            return ok & (z > 0) & (z < d)
        ok = -(X[2] * X[3]) > 0
        q = X / X[3]
        ok &= -q[2] < d
        z = P[2, 0] * q[0] + P[2, 1] * q[1] + P[2, 2] * q[2] + P[2, 3] * q[3]
        return ok & (-z > 0) & (-z < d)


def test_pose_mirror_exact(oracle_mod):
    rng = np.random.default_rng(7)
    P0 = np.hstack([np.eye(3), np.zeros((3, 1))])
    n_checked = 0
    for trial in range(24):
        R = _rot(rng)
        t = rng.standard_normal(3)
        t /= np.linalg.norm(t)
        Pp = np.hstack([R + 0.0, (t + 0.0).reshape(3, 1)])
        Pm = np.hstack([R + 0.0, (0.0 - (t + 0.0)).reshape(3, 1)])
        k = 4000
        scale = [0.05, 0.5, 2.0][trial % 3]
        x1 = rng.standard_normal((2, k)) * scale
        x2 = x1 + rng.standard_normal((2, k)) * scale * 0.3
        if trial % 4 == 3:  # exact duplicates / collinear rows
            x2[:, : k // 4] = x1[:, : k // 4]
        X = oracle_mod.triangulate(P0, Pp, x1, x2)
        Xm = oracle_mod.triangulate(P0, Pm, x1, x2)
        mirrored = np.vstack([X[0], X[1], X[2], -X[3]])
        sigma = np.where(np.signbit(Xm[3]) == np.signbit(mirrored[3]), 1.0, -1.0)
        np.testing.assert_array_equal(Xm, sigma * mirrored)
        for d in (50.0, 2.0):
            np.testing.assert_array_equal(_tests(X, Pp, d, True), _tests(Xm, Pm, d, False))
        n_checked += k
    assert n_checked == 96000
