"""Drop-in pose_estimation_module (dropin/pose_estimation_module.py) against
scripts/pose_estimation_module.py semantics: quaternion branches, TUM lines,
marker/camera relative transforms, velocity."""
import math

import numpy as np
import pytest

from droplet_visual_odometry_amd import transformations as tr
from droplet_visual_odometry_amd.dropin import pose_estimation_module as pem


def _same_rotation(q1, q2):
    q1, q2 = np.asarray(q1), np.asarray(q2)
    return np.allclose(q1, q2, atol=1e-12) or np.allclose(q1, -q2, atol=1e-12)


@pytest.mark.parametrize("R", [
    tr.euler_matrix(0.1, 0.2, 0.3)[:3, :3],                 # trace > 0
    tr.euler_matrix(math.pi - 0.1, 0.05, 0.02)[:3, :3],     # R00 largest
    tr.euler_matrix(0.02, math.pi - 0.1, 0.05)[:3, :3],     # R11 largest
    tr.euler_matrix(0.05, 0.02, math.pi - 0.1)[:3, :3] @ tr.euler_matrix(math.pi, 0, 0)[:3, :3],  # R22 largest
])
def test_rotation_matrix_to_quaternion_branches(R):
    q = pem.rotation_matrix_to_quaternion(R)
    assert _same_rotation(q, tr.quaternion_from_matrix(np.block([[R, np.zeros((3, 1))], [np.zeros((1, 3)), 1]])))
    T = np.eye(4)
    T[:3, :3] = R
    assert pem.quaternion_from_transformation_matrix(T) == q


def test_branch_coverage_is_real():
    traces = [np.trace(tr.euler_matrix(*a)[:3, :3]) for a in [(0.1, 0.2, 0.3), (math.pi - 0.1, 0.05, 0.02)]]
    assert traces[0] > 0 and traces[1] <= 0


def test_transformation_from_translation_quaternion():
    q = tr.quaternion_from_euler(0.1, -0.2, 0.3)
    T = pem.transformation_from_translation_quaternion([1, 2, 3], q)
    np.testing.assert_allclose(T[:3, :3], tr.euler_matrix(0.1, -0.2, 0.3)[:3, :3], atol=1e-12)
    assert pem.translation_from_transformation_matrix(T) == [1, 2, 3]


def test_marker_and_camera_relative():
    rng = np.random.default_rng(1)
    A = tr.euler_matrix(*rng.uniform(-1, 1, 3))
    A[:3, 3] = rng.uniform(-1, 1, 3)
    B = tr.euler_matrix(*rng.uniform(-1, 1, 3))
    B[:3, 3] = rng.uniform(-1, 1, 3)
    np.testing.assert_allclose(A @ pem.get_marker_to_marker_transformation(A, B), B, atol=1e-12)
    np.testing.assert_allclose(pem.get_camera_to_camera_transformation(A, B) @ B, A, atol=1e-12)


def test_tum_line_format(tmp_path):
    f = tmp_path / "vo.txt"
    pem.write_to_output_file(str(f), 1.5, [1, 2.25, np.float64(3)], [0.0, 0.0, 0.0, 1.0])
    pem.write_to_output_file(str(f), 2, np.array([0.5, 0.5, 0.5]), np.array([0.1, 0.2, 0.3, 0.4]))
    assert f.read_text() == "1.5 1 2.25 3.0 0.0 0.0 0.0 1.0 \n2 0.5 0.5 0.5 0.1 0.2 0.3 0.4 \n"
    pem.clear_txt_file_contents(str(f))
    assert f.read_text() == ""


def test_velocity_elementwise():
    T = tr.euler_matrix(0.1, 0.2, 0.3)
    T[:3, 3] = [0.2, -0.4, 0.6]
    v = pem.get_velocity_between_timestamps(T, 10.0, 10.5)
    np.testing.assert_allclose(v[:3, 3], [0.4, -0.8, 1.2])
    np.testing.assert_allclose(v[:3, :3], T[:3, :3] / 0.5)
    np.testing.assert_array_equal(v[3], [0, 0, 0, 1])


def test_gt_vo_difference_files(tmp_path):
    gt = tmp_path / "gt.txt"
    vo = tmp_path / "vo.txt"
    qg = tr.quaternion_from_euler(0.1, 0.2, 0.3)
    qv = tr.quaternion_from_euler(0.15, 0.2, 0.25)
    for f, q in ((gt, qg), (vo, qv)):
        for ts in (1.0, 2.0):
            pem.write_to_output_file(str(f), ts, [0, 0, 0], q)
    d = pem.get_gt_vo_difference(str(gt), str(vo))
    np.testing.assert_allclose(d, [0.05, 0.0, -0.05], atol=1e-12)
    out = tmp_path / "diff.txt"
    pem.write_gt_vo_difference_to_file(str(gt), str(vo), str(out))
    assert out.read_text().startswith("at timestamp 1.0 the gt vo euler angle difference is ")


def _tf_log():
    import json
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tf_log_transforms.json")
    return json.load(open(path))["transforms"]


def test_real_tf_log_round_trips_through_the_pose_helpers():
    """The 454 ROS tf transforms the reference's author logged
    (scripts/back_up_files/log.txt, transcribed by
    tests/golden/make_tf_log_kats.py): STag marker poses in the camera frame,
    base_link and the AHRS orientation.  For each one,
    transformation_from_translation_quaternion (pem:15-23, tf.quaternion_matrix)
    followed by quaternion_from_transformation_matrix (pem:60-65 -> the trace
    branches of pem:31-57) returns the logged (x, y, z, w) up to sign, and
    translation_from_transformation_matrix (pem:26-28) the logged translation
    exactly.  Every trace branch the real data reaches is exercised."""
    logs = _tf_log()
    assert len(logs) == 454
    branches = set()
    for e in logs:
        t, q = e["t"], np.array(e["q"])
        assert abs(np.linalg.norm(q) - 1) < 1e-9, e["line"]  # ROS publishes unit quaternions (to print precision)
        T = pem.transformation_from_translation_quaternion(t, q)
        np.testing.assert_allclose(T[:3, :3] @ T[:3, :3].T, np.eye(3), atol=1e-9)
        assert pem.translation_from_transformation_matrix(T) == t
        got = np.array(pem.quaternion_from_transformation_matrix(T))
        assert _same_rotation_tol(got, q, 1e-9), (e["line"], got, q)
        R = T[:3, :3]
        tr_ = np.trace(R)
        branches.add("trace" if tr_ > 0 else ("r00" if R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]
                                               else ("r11" if R[1, 1] > R[2, 2] else "r22")))
    assert {"trace", "r00"} <= branches, branches


def _same_rotation_tol(q1, q2, tol):
    return np.allclose(q1, q2, atol=tol) or np.allclose(q1, -q2, atol=tol)


def test_real_tf_log_marker_to_marker_motion_is_rigid():
    """Consecutive logged poses of one marker composed the way the harness does
    (get_marker_to_marker_transformation, pem: marker pose at t-1 inverted times
    the pose at t) give proper rigid motions whose quaternion round-trips too."""
    logs = [e for e in _tf_log() if e["child_frame_id"] == "/ar_marker_0"]
    Ts = [pem.transformation_from_translation_quaternion(e["t"], e["q"]) for e in logs]
    for a, b in zip(Ts, Ts[1:]):
        M = pem.get_marker_to_marker_transformation(a, b)
        R = M[:3, :3]
        np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-9)
        assert abs(np.linalg.det(R) - 1) < 1e-9
        q = pem.quaternion_from_transformation_matrix(M)
        M2 = pem.transformation_from_translation_quaternion(pem.translation_from_transformation_matrix(M),
                                                            np.array(q) / np.linalg.norm(q))
        np.testing.assert_allclose(M2, M, atol=1e-9)
