"""The restated Gohlke `transformations` / ROS tf helpers (transformations.py),
pinned by the published doctest values of transformations.py (C. Gohlke,
2006-2017 releases: euler_matrix(1, 2, 3, 'syxz') row-0 sum, quaternion
conventions) and by identities over all 24 axis sequences."""
import math

import numpy as np
import pytest

from droplet_visual_odometry_amd import transformations as tr


def Rx(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])


def Ry(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def Rz(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def test_published_doctest_values():
    R = tr.euler_matrix(1, 2, 3, "syxz")
    assert np.allclose(np.sum(R[0]), -1.34786452)
    R = tr.euler_matrix(1, 2, 3, (0, 1, 0, 1))
    assert np.allclose(np.sum(R[0]), -0.383436184)


@pytest.mark.parametrize("axes", sorted(tr._AXES2TUPLE))
def test_euler_round_trip_all_axes(axes):
    rng = np.random.default_rng(hash(axes) % 2 ** 32)
    for _ in range(20):
        ang = rng.uniform(-math.pi, math.pi, 3)
        R0 = tr.euler_matrix(*ang, axes=axes)
        R1 = tr.euler_matrix(*tr.euler_from_matrix(R0, axes), axes=axes)
        np.testing.assert_allclose(R0, R1, atol=1e-12)
        np.testing.assert_allclose(R0[:3, :3] @ R0[:3, :3].T, np.eye(3), atol=1e-12)


def test_static_and_rotating_conventions():
    a, b, c = 0.3, -0.7, 1.1
    np.testing.assert_allclose(tr.euler_matrix(a, b, c, "sxyz")[:3, :3], Rz(c) @ Ry(b) @ Rx(a), atol=1e-14)
    np.testing.assert_allclose(tr.euler_matrix(a, b, c, "rxyz")[:3, :3], Rx(a) @ Ry(b) @ Rz(c), atol=1e-14)


def test_reference_rxyz_to_sxyz_rebuild():
    """D4: visual_odometry_v3.py:334-341 reads angles with 'rxyz' and rebuilds with
    'sxyz', i.e. R = Rx(a)Ry(b)Rz(c) becomes Rz(c)Ry(b)Rx(a) — kept as is."""
    a, b, c = 0.05, -0.02, 0.11
    R = Rx(a) @ Ry(b) @ Rz(c)
    ang = tr.euler_from_matrix(R, "rxyz")
    np.testing.assert_allclose(ang, (a, b, c), atol=1e-14)
    M = tr.euler_matrix(*ang, axes="sxyz")[:3, :3]
    np.testing.assert_allclose(M, Rz(c) @ Ry(b) @ Rx(a), atol=1e-14)
    assert not np.allclose(M, R, atol=1e-6)


def test_gimbal_lock_branch():
    R = tr.euler_matrix(0.4, math.pi / 2, 0.0, "sxyz")
    ang = tr.euler_from_matrix(R, "sxyz")
    np.testing.assert_allclose(tr.euler_matrix(*ang, axes="sxyz"), R, atol=1e-12)


def test_translation_helpers():
    T = tr.translation_matrix([1.0, -2.0, 3.5])
    np.testing.assert_array_equal(tr.translation_from_matrix(T), [1.0, -2.0, 3.5])
    np.testing.assert_array_equal(tr.identity_matrix(), np.eye(4))


def test_tf_quaternion_order_xyzw():
    # tf order (x, y, z, w): rotation of 0.123 rad about x.
    q = [math.sin(0.0615), 0.0, 0.0, math.cos(0.0615)]
    np.testing.assert_allclose(tr.quaternion_matrix(q)[:3, :3], Rx(0.123), atol=1e-14)
    np.testing.assert_allclose(tr.quaternion_from_matrix(tr.quaternion_matrix(q)), q, atol=1e-14)
    np.testing.assert_allclose(tr.euler_from_quaternion(q), (0.123, 0.0, 0.0), atol=1e-14)
    np.testing.assert_allclose(tr.quaternion_matrix([0, 0, 0, 0]), np.eye(4))


def test_quaternion_euler_round_trip():
    rng = np.random.default_rng(7)
    for _ in range(50):
        ang = rng.uniform(-3, 3, 3)
        q = tr.quaternion_from_euler(*ang)
        assert abs(np.linalg.norm(q) - 1) < 1e-12
        np.testing.assert_allclose(tr.quaternion_matrix(q), tr.euler_matrix(*ang), atol=1e-12)


def test_unknown_axes_raise():
    with pytest.raises(KeyError):
        tr.euler_matrix(0, 0, 0, "abc")
