"""SIFT_create().detectAndCompute on the GPU (dvo_sift_detect_and_compute)
against the oracle's restatement of OpenCV 4.x SIFT (oracle/sift.cpp): the
detector of the reference's sift / knn_sift / flann modes
(visual_odometry_v3.py:99-103, :373).  Keypoints (every field, in
removeDuplicatedSorted order) and the 128 descriptor values bit-identical;
then the knn_sift and flann modes end to end through the drop-in
(visual_odometry_calculations, v3:384-408).  Parity against OpenCV itself is
unpinned (no cv2 here)."""
import os
import sys

import numpy as np
import pytest

from conftest import synth_frames

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _check(gpu_ctx, oracle_mod, img):
    from droplet_visual_odometry_amd import ops
    kg, dg = ops.sift_detect_and_compute(img, ctx=gpu_ctx)
    ko, do = oracle_mod.sift_detect_and_compute(img)
    assert len(kg) == len(ko)
    np.testing.assert_array_equal(kg.view(np.uint8), ko.view(np.uint8))
    np.testing.assert_array_equal(dg.view(np.uint32), do.view(np.uint32))
    return len(kg)


def test_sift_synthetic_frames(gpu_ctx, oracle_mod):
    frames, _ = synth_frames(640, 480, range(2))
    for f in frames:
        assert _check(gpu_ctx, oracle_mod, f) > 500


@pytest.mark.parametrize("wh", [(8, 8), (40, 30), (97, 61), (161, 97), (333, 211)])
def test_sift_small_and_odd_sizes(gpu_ctx, oracle_mod, wh):
    w, h = wh
    rng = np.random.default_rng(w * 31 + h)
    img = rng.integers(0, 256, (h, w), dtype=np.uint8)
    img = np.clip(img.astype(np.int32) // 2 + np.add.outer(np.arange(h) * 3, np.arange(w) * 2) % 128, 0, 255)
    _check(gpu_ctx, oracle_mod, np.ascontiguousarray(img.astype(np.uint8)))


def test_sift_blank_frame(gpu_ctx, oracle_mod):
    assert _check(gpu_ctx, oracle_mod, np.full((120, 160), 90, np.uint8)) == 0


def test_sift_cv_surface(gpu_ctx):
    from droplet_visual_odometry_amd import cv
    frames, _ = synth_frames(640, 480, range(1))
    kps, desc = cv.xfeatures2d.SIFT_create().detectAndCompute(frames[0], None)
    assert len(kps) == len(desc) and desc.dtype == np.float32 and desc.shape[1] == 128
    assert np.all(desc == np.round(desc)) and desc.min() >= 0 and desc.max() <= 255
    assert all(k.class_id == -1 for k in kps[:10])
    xs = cv.KeyPoint_convert(kps)
    assert np.all(np.diff(xs[:, 0]) >= 0)  # removeDuplicatedSorted: x ascending first


def _yaml(K):
    d = ", ".join(repr(float(v)) for v in K.ravel())
    return (f"camera_matrix:\n  rows: 3\n  cols: 3\n  data: [{d}]\n"
            "distortion_coefficients:\n  rows: 1\n  cols: 5\n  data: [0.0, 0.0, 0.0, 0.0, 0.0]\n")


@pytest.mark.parametrize("mode", ["knn_sift", "flann"])
def test_dropin_sift_modes_end_to_end(gpu_ctx, oracle_mod, tmp_path, mode):
    """visual_odometry_calculations in the k-NN SIFT modes: SIFT on both
    frames, knnMatch(k=2) (BFMatcher L1 or the FLANN kd-forest, its theRNG
    state carried from pair to pair), the 0.75 ratio
    test (v3:223-228), findEssentialMat / recoverPose on the kept keypoints;
    E bit-identical to the oracle run of the same chain."""
    from droplet_visual_odometry_amd.synth import MARKER_LEN, marker_corners
    sys.path.insert(0, os.path.join(ROOT, "droplet_visual_odometry_amd", "dropin"))
    try:
        import visual_odometry_v3 as v3
    finally:
        sys.path.pop(0)
    frames, K = synth_frames(640, 480, range(3))
    y = tmp_path / "cal.yaml"
    y.write_text(_yaml(K))
    vo = v3.VisualOdometry(mode=mode, calibration_file_path=str(y), controlled=True, real_marker_length=MARKER_LEN)
    T = vo.robot_curr_position
    from droplet_visual_odometry_amd import cv
    cv.setRNGSeed(0)  # the harness process's cv::theRNG(), carried across the pairs
    state = oracle_mod.THE_RNG_SEED
    for i in range(2):
        T, rel = vo.visual_odometry_calculations(frames[i], frames[i + 1], T, marker_corners(i, K),
                                                 marker_corners(i + 1, K))
        k1, d1 = oracle_mod.sift_detect_and_compute(frames[i])
        k2, d2 = oracle_mod.sift_detect_and_compute(frames[i + 1])
        if mode == "flann":
            idx, dist, state = oracle_mod.flann_knn(d1, d2, 2, trees=5, checks=50, rng_state=state)
            dist = np.sqrt(dist.astype(np.float32))
        else:
            idx, dist = oracle_mod.bf_knn_float(d1, d2, 2, 0)
        keep = [q for q in range(len(d1)) if float(dist[q, 0]) < 0.75 * float(dist[q, 1])]
        p1 = np.stack([k1["x"][keep], k1["y"][keep]], 1).astype(np.float64)
        p2 = np.stack([k2["x"][idx[keep, 0]], k2["y"][idx[keep, 0]]], 1).astype(np.float64)
        E, _, _ = oracle_mod.find_essential(p1, p2, K)
        np.testing.assert_array_equal(vo.essential_matrix, E)
        assert np.all(np.isfinite(rel))
