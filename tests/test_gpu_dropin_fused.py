"""The drop-in's fused pair path (D7, dvo_stream_pair / ops.PairStream):
visual_odometry_calculations with the stock ORB / BFMatcher(NORM_HAMMING,
crossCheck) runs detect -> match -> findEssentialMat -> recoverPose in one
library call and then the same host tail as the operator-by-operator path
(visual_odometry_v3.py:384-408, driven as trajectory_evaluation_dual_process.py:
151-166 drives it).  The two paths must give identical 4x4s, E and P_prev (bit
for bit), whether or not the previous frame's device features are reused, and
a failing pair must raise where the operator path raises."""
import os
import sys

import numpy as np
import pytest

from conftest import synth_frames

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _v3():
    sys.path.insert(0, os.path.join(ROOT, "droplet_visual_odometry_amd", "dropin"))
    try:
        import visual_odometry_v3 as v3
    finally:
        sys.path.pop(0)
    return v3


def _make(v3, K, tmp_path, slow, nfeatures=None):
    from droplet_visual_odometry_amd.synth import MARKER_LEN
    d = ", ".join(repr(float(v)) for v in K.ravel())
    y = tmp_path / ("slow.yaml" if slow else "fused.yaml")
    y.write_text(f"camera_matrix:\n  rows: 3\n  cols: 3\n  data: [{d}]\n"
                 "distortion_coefficients:\n  rows: 1\n  cols: 5\n  data: [0.0, 0.0, 0.0, 0.0, 0.0]\n")

    class OperatorByOperator(v3.VisualOdometry):  # an overridden per-pair method disables the fused path
        def compute_current_image_elements(self, input_image):
            return super().compute_current_image_elements(input_image)

    cls = OperatorByOperator if slow else v3.VisualOdometry
    vo = cls(mode="orb", calibration_file_path=str(y), controlled=True, real_marker_length=MARKER_LEN)
    if nfeatures:
        vo.feature_detector.setMaxFeatures(nfeatures)
    return vo


@pytest.mark.parametrize("W,H,NF", [(640, 480, None), (1280, 720, 2000)])
def test_fused_equals_operator_path(gpu_ctx, tmp_path, W, H, NF):
    from droplet_visual_odometry_amd.synth import marker_corners
    v3 = _v3()
    frames, K = synth_frames(W, H, range(8))
    corners = [marker_corners(i, K) for i in range(8)]
    fused, slow = _make(v3, K, tmp_path, False, NF), _make(v3, K, tmp_path, True, NF)
    # consecutive pairs (device features reused), a jump (both frames detected), a repeat
    seq = [(0, 1), (1, 2), (2, 3), (4, 5), (5, 6), (5, 6), (6, 7), (0, 7)]
    Tf, Ts = fused.robot_curr_position, slow.robot_curr_position
    for a, b in seq:
        Tf, rf = fused.visual_odometry_calculations(frames[a], frames[b], Tf, corners[a], corners[b])
        Ts, rs = slow.visual_odometry_calculations(frames[a], frames[b], Ts, corners[a], corners[b])
        np.testing.assert_array_equal(rf, rs)
        np.testing.assert_array_equal(Tf, Ts)
        np.testing.assert_array_equal(fused.essential_matrix, slow.essential_matrix)
        np.testing.assert_array_equal(fused.previous_projection_matrix, slow.previous_projection_matrix)
    assert fused._pair_engine is not None and slow._pair_engine is None
    assert len(fused.frame_translations) == len(seq) == len(slow.frame_translations)
    for x, y in zip(fused.projection_matrix_list, slow.projection_matrix_list):
        np.testing.assert_array_equal(x, y)


def test_fused_failing_pair_raises_like_operator_path(gpu_ctx, tmp_path):
    from droplet_visual_odometry_amd import cv
    from droplet_visual_odometry_amd.synth import marker_corners
    v3 = _v3()
    frames, K = synth_frames(640, 480, range(3))
    blank = np.zeros_like(frames[0])
    c = [marker_corners(i, K) for i in range(3)]
    for slow in (False, True):
        vo = _make(v3, K, tmp_path, slow)
        T, _ = vo.visual_odometry_calculations(frames[0], frames[1], vo.robot_curr_position, c[0], c[1])
        with pytest.raises(cv.error):
            vo.visual_odometry_calculations(frames[1], blank, T, c[1], c[2])
        # and the stream recovers: the next good pair (the previous frame's features re-detected)
        T2, _ = vo.visual_odometry_calculations(frames[1], frames[2], T, c[1], c[2])
        if slow:
            np.testing.assert_array_equal(T2, T2_fused)
        else:
            T2_fused = T2


def test_fused_opencv32(gpu_ctx, tmp_path, monkeypatch):
    """OpenCV 3.2 semantics (ORB pyramid / retainBest, 3.x cross check) on the fused path."""
    from droplet_visual_odometry_amd import cv
    from droplet_visual_odometry_amd.synth import marker_corners
    monkeypatch.setattr(cv, "OPENCV_SEMANTICS", "3.2")
    v3 = _v3()
    frames, K = synth_frames(640, 480, range(4))
    c = [marker_corners(i, K) for i in range(4)]
    fused, slow = _make(v3, K, tmp_path, False), _make(v3, K, tmp_path, True)
    assert fused.feature_detector.opencv == "3.2" and fused.bf.legacy_crosscheck
    Tf, Ts = fused.robot_curr_position, slow.robot_curr_position
    for a in range(3):
        Tf, _ = fused.visual_odometry_calculations(frames[a], frames[a + 1], Tf, c[a], c[a + 1])
        Ts, _ = slow.visual_odometry_calculations(frames[a], frames[a + 1], Ts, c[a], c[a + 1])
        np.testing.assert_array_equal(Tf, Ts)
    assert fused._pair_engine is not None


def test_pair_stream_record_equals_batched_stream(gpu_ctx):
    """ops.PairStream's record: R, t, E, counts equal the batched stream's for the same pair
    (n_hypotheses aside: the per-call RANSAC schedule takes one round)."""
    import torch
    from droplet_visual_odometry_amd import ops
    from droplet_visual_odometry_amd.stream import FrameStream
    frames, K = synth_frames(1280, 720, range(4))
    ps = ops.PairStream(1280, 720, K, nfeatures=2000, ctx=gpu_ctx)
    fs = FrameStream(1280, 720, K, nfeatures=2000, max_frames=4, ctx=gpu_ctx)
    rec = fs.process(torch.from_numpy(frames).cuda())
    fs.sync()
    want = FrameStream.records_numpy(rec, 3)
    for p in range(3):
        got = ps.pair(frames[p], frames[p + 1], reuse_prev=p > 0)
        for k in ("R", "t", "E", "n_kp_prev", "n_kp_cur", "n_matches", "n_inliers", "n_good", "ransac_iters", "status",
                  "n_models"):
            np.testing.assert_array_equal(got[k], want[p][k], err_msg=k)
    with pytest.raises(Exception):
        ops.PairStream(640, 480, K, ctx=gpu_ctx).pair(None, frames[0][:480, :640], reuse_prev=True)
    ps.close()
    fs.close()
