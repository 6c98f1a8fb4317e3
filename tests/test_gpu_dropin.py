"""The drop-in VisualOdometry driven the way trajectory_evaluation_dual_process.py
drives the reference (dual:151-166: ros_img_msg_to_opencv_image on each
message, i.e. BGR->gray + undistort with the optimal new camera matrix, then
visual_odometry_calculations with the previous absolute pose and the marker
corners), over a synthetic 640x480 usb_raw stream, against the oracle
(undistort + pair path + the host pose-tail restatement).  R, t, E bit-exact; the 4x4 poses
(numpy / libm on both sides, same operation order) within 1e-12."""
import os
import sys
import types

import numpy as np
import pytest

from conftest import synth_frames

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _yaml(K):
    d = ", ".join(repr(float(v)) for v in K.ravel())
    return (f"camera_matrix:\n  rows: 3\n  cols: 3\n  data: [{d}]\n"
            "distortion_coefficients:\n  rows: 1\n  cols: 5\n  data: [0.0, 0.0, 0.0, 0.0, 0.0]\n")


def test_visual_odometry_replay(gpu_ctx, oracle_mod, tmp_path):
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    sys.path.insert(0, os.path.join(ROOT, "droplet_visual_odometry_amd", "dropin"))
    try:
        import visual_odometry_v3 as v3
    finally:
        sys.path.pop(0)
    frames, K = synth_frames(640, 480, range(5))
    y = tmp_path / "cal.yaml"
    y.write_text(_yaml(K))
    vo = v3.VisualOdometry(mode="orb", calibration_file_path=str(y), controlled=True, real_marker_length=MARKER_LEN)
    msgs = [types.SimpleNamespace(data=np.repeat(f[..., None], 3, axis=2).tobytes(), height=480, width=640)
            for f in frames]
    corners = [marker_corners(i, K) for i in range(5)]
    # the reference undistorts every frame with new_K = getOptimalNewCameraMatrix(K, 0, size, 1)
    # (v3:117-120; zero distortion still rescales by (w-1)/w) and keeps the original K for E / pose
    new_K = oracle_mod.get_optimal_new_camera_matrix(K, np.zeros(5), 640, 480, 1.0)
    und = [oracle_mod.undistort(f, K, np.zeros(5), new_K)[0] for f in frames]
    T_vo = vo.robot_curr_position
    P = K @ np.hstack((np.eye(3), np.zeros((3, 1))))
    T_ref = np.eye(4)
    for i in range(1, 5):
        prev = vo.ros_img_msg_to_opencv_image(msgs[i - 1], "usb_raw")
        cur = vo.ros_img_msg_to_opencv_image(msgs[i], "usb_raw")
        np.testing.assert_array_equal(prev, und[i - 1])
        np.testing.assert_array_equal(cur, und[i])
        T_vo, rel = vo.visual_odometry_calculations(prev, cur, T_vo, corners[i - 1], corners[i])
        ref = oracle_mod.pair_pose(und[i - 1], und[i], K, 500)
        np.testing.assert_array_equal(vo.essential_matrix, ref["E"])
        P, T_rel, T_ref = oracle_mod.pose_tail(K, ref["R"], ref["t_unit"], corners[i - 1], corners[i], MARKER_LEN,
                                               P, T_ref)
        np.testing.assert_array_equal(vo.previous_projection_matrix, P)
        np.testing.assert_allclose(rel, T_rel, rtol=0, atol=1e-12)
        np.testing.assert_allclose(T_vo, T_ref, rtol=0, atol=1e-12)
    assert len(vo.frame_translations) == 4 and len(vo.projection_matrix_list) == 4


def test_array_backed_matches_equal_object_path(gpu_ctx, frames_640):
    """The drop-in's ORB branch on cv.DMatches / cv.KeyPoints (stable argsort +
    index gather) returns what the reference's object loop returns
    (sorted(matches, key=distance), then prev_kp[m.queryIdx], cur_kp[m.trainIdx],
    v3:219-238) on plain lists of the same objects."""
    from droplet_visual_odometry_amd import cv
    sys.path.insert(0, os.path.join(ROOT, "droplet_visual_odometry_amd", "dropin"))
    try:
        import visual_odometry_v3 as v3
    finally:
        sys.path.pop(0)
    frames, _ = frames_640
    orb = cv.ORB_create(nfeatures=1000)
    kp0, d0 = orb.detectAndCompute(frames[0], None)
    kp1, d1 = orb.detectAndCompute(frames[1], None)
    assert isinstance(kp0, cv.KeyPoints) and len(kp0) == len(d0)
    bf = cv.BFMatcher(normType=cv.NORM_HAMMING, crossCheck=True)
    me = types.SimpleNamespace(mode="orb", bf=bf)
    matches, top_prev, top_cur = v3.VisualOdometry.get_matches_between_two_frames(me, kp0, d0, kp1, d1)
    ref = sorted(list(bf.match(d0, d1)), key=lambda x: x.distance)
    assert [(m.queryIdx, m.trainIdx, m.distance) for m in matches] == \
        [(m.queryIdx, m.trainIdx, m.distance) for m in ref]
    assert [k.pt for k in top_prev] == [kp0[m.queryIdx].pt for m in ref]
    assert [k.pt for k in top_cur] == [kp1[m.trainIdx].pt for m in ref]
    # lists of plain KeyPoint objects take the reference's loop and agree
    _, lp, lc = v3.VisualOdometry.get_matches_between_two_frames(me, list(kp0), d0, list(kp1), d1)
    np.testing.assert_array_equal(cv.KeyPoint_convert(lp), cv.KeyPoint_convert(top_prev))
    np.testing.assert_array_equal(cv.KeyPoint_convert(lc), cv.KeyPoint_convert(top_cur))
    # the lazily drawn keypoint image (v3:375) is the eager one
    vo = types.SimpleNamespace(feature_detector=orb, _features=v3._FeatureCache())
    kps, desc, drawn = v3.VisualOdometry.compute_current_image_elements(vo, frames[2])
    np.testing.assert_array_equal(np.asarray(drawn),
                                  cv.drawKeypoints(frames[2], kps, None, color=(0, 255, 0), flags=0))
    assert drawn.shape == (480, 640, 3)
