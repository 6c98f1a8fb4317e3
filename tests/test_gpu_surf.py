"""xfeatures2d.SURF_create(400).detectAndCompute on the GPU
(dvo_surf_detect_and_compute) against the oracle's restatement of
opencv_contrib SURF (oracle/surf.cpp): the detector of the reference's 'surf'
mode (visual_odometry_v3.py:103-106, :373).  Keypoints (every field, in
KeypointGreater order) and the 64 descriptor values bit-identical; then the
surf mode end to end through the drop-in (knnMatch + 0.75 ratio test,
v3:212-228).  Parity against OpenCV itself is unpinned (no cv2 here)."""
import os
import sys

import numpy as np
import pytest

from conftest import synth_frames

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _check(gpu_ctx, oracle_mod, img, thr=400.0):
    from droplet_visual_odometry_amd import ops
    kg, dg = ops.surf_detect_and_compute(img, thr, ctx=gpu_ctx)
    ko, do = oracle_mod.surf_detect_and_compute(img, thr)
    assert len(kg) == len(ko)
    np.testing.assert_array_equal(kg.view(np.uint8), ko.view(np.uint8))
    np.testing.assert_array_equal(dg.view(np.uint32), do.view(np.uint32))
    return len(kg)


def test_surf_synthetic_frames(gpu_ctx, oracle_mod):
    frames, _ = synth_frames(640, 480, range(2))
    for f in frames:
        assert _check(gpu_ctx, oracle_mod, f) > 500


def test_surf_1280x720(gpu_ctx, oracle_mod):
    frames, _ = synth_frames(1280, 720, range(1))
    assert _check(gpu_ctx, oracle_mod, frames[0]) > 1000


@pytest.mark.parametrize("thr", [0.0, 100.0, 5000.0])
def test_surf_thresholds(gpu_ctx, oracle_mod, thr):
    frames, _ = synth_frames(320, 240, range(1))
    _check(gpu_ctx, oracle_mod, frames[0], thr)


@pytest.mark.parametrize("wh", [(8, 8), (40, 30), (97, 61), (161, 97), (333, 211)])
def test_surf_small_and_odd_sizes(gpu_ctx, oracle_mod, wh):
    w, h = wh
    rng = np.random.default_rng(w * 31 + h)
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    img = np.clip(img.astype(np.int32) // 2 + np.add.outer(np.arange(h) * 3, np.arange(w) * 2) % 128, 0, 255)
    _check(gpu_ctx, oracle_mod, np.ascontiguousarray(img.astype(np.uint8)), 100.0)


def test_surf_blank_frame(gpu_ctx, oracle_mod):
    assert _check(gpu_ctx, oracle_mod, np.full((120, 160), 90, np.uint8)) == 0


def test_surf_cv_surface(gpu_ctx):
    from droplet_visual_odometry_amd import cv
    frames, _ = synth_frames(640, 480, range(1))
    kps, desc = cv.xfeatures2d.SURF_create(400).detectAndCompute(frames[0], None)
    assert len(kps) == len(desc) and desc.dtype == np.float32 and desc.shape[1] == 64
    np.testing.assert_allclose(np.linalg.norm(desc, axis=1), 1.0, rtol=1e-5)
    assert all(k.class_id in (-1, 1) for k in kps[:50])
    resp = np.array([k.response for k in kps])
    assert np.all(np.diff(resp) <= 0)  # KeypointGreater: response descending first


def _yaml(K):
    d = ", ".join(repr(float(v)) for v in K.ravel())
    return (f"camera_matrix:\n  rows: 3\n  cols: 3\n  data: [{d}]\n"
            "distortion_coefficients:\n  rows: 1\n  cols: 5\n  data: [0.0, 0.0, 0.0, 0.0, 0.0]\n")


def test_dropin_surf_mode_end_to_end(gpu_ctx, oracle_mod, tmp_path):
    """visual_odometry_calculations in the surf mode: SURF_create(400) on both
    frames, BFMatcher(NORM_L1).knnMatch(k=2) (v3:215), the 0.75 ratio test,
    findEssentialMat / recoverPose on the kept keypoints; E bit-identical to
    the oracle run of the same chain."""
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    sys.path.insert(0, os.path.join(ROOT, "droplet_visual_odometry_amd", "dropin"))
    try:
        import visual_odometry_v3 as v3
    finally:
        sys.path.pop(0)
    frames, K = synth_frames(640, 480, range(3))
    y = tmp_path / "cal.yaml"
    y.write_text(_yaml(K))
    vo = v3.VisualOdometry(mode="surf", calibration_file_path=str(y), controlled=True, real_marker_length=MARKER_LEN)
    T = vo.robot_curr_position
    for i in range(2):
        T, rel = vo.visual_odometry_calculations(frames[i], frames[i + 1], T, marker_corners(i, K),
                                                 marker_corners(i + 1, K))
        k1, d1 = oracle_mod.surf_detect_and_compute(frames[i], 400.0)
        k2, d2 = oracle_mod.surf_detect_and_compute(frames[i + 1], 400.0)
        idx, dist = oracle_mod.bf_knn_float(d1, d2, 2, 0)
        keep = [q for q in range(len(d1)) if float(dist[q, 0]) < 0.75 * float(dist[q, 1])]
        p1 = np.stack([k1["x"][keep], k1["y"][keep]], 1).astype(np.float64)
        p2 = np.stack([k2["x"][idx[keep, 0]], k2["y"][idx[keep, 0]]], 1).astype(np.float64)
        E, _, _ = oracle_mod.find_essential(p1, p2, K)
        np.testing.assert_array_equal(vo.essential_matrix, E)
        assert np.all(np.isfinite(rel))
