"""Host-side pieces of the cv2 surface and of the drop-in VisualOdometry that
need no GPU: colour conversion, keypoint conversion, error behaviour, YAML
parsing, ROS message decoding, the pose composition helpers."""
import os
import sys
import types

import numpy as np
import pytest

from droplet_visual_odometry_amd import cv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bgr2gray_fixed_point():
    px = np.array([[[0, 0, 0], [255, 255, 255], [10, 200, 30], [255, 0, 0], [0, 0, 255], [1, 2, 3]]], np.uint8)
    got = cv.cvtColor(px, cv.COLOR_BGR2GRAY)
    want = [(int(b) * 1868 + int(g) * 9617 + int(r) * 4899 + 8192) >> 14 for b, g, r in px[0]]
    assert got[0].tolist() == want
    assert want[:2] == [0, 255]
    assert cv.cvtColor(got, cv.COLOR_BGR2GRAY).tolist() == got.tolist()


def test_keypoint_convert_and_dmatch():
    kps = [cv.KeyPoint(1.5, 2.5, 31), cv.KeyPoint(3.0, 4.0, 31)]
    np.testing.assert_array_equal(cv.KeyPoint_convert(kps), np.array([[1.5, 2.5], [3.0, 4.0]], np.float32))
    assert cv.KeyPoint_convert([]).shape == (0, 2)
    m = cv.DMatch(1, 2, 0, 3.0)
    assert m[0] is m and m.queryIdx == 1 and m.trainIdx == 2 and m.distance == 3.0


def test_unsupported_modes_raise_cv_error():
    with pytest.raises(cv.error):
        cv.ORB_create(nlevels=4)
    with pytest.raises(cv.error):
        cv.BFMatcher(cv.NORM_L2).match(np.zeros((2, 32), np.uint8), np.zeros((2, 32), np.uint8))
    with pytest.raises(cv.error):
        cv.findEssentialMat(np.zeros((5, 2)), np.zeros((5, 2)), np.eye(3), method=cv.LMEDS)
    with pytest.raises(cv.error):
        cv.recoverPose(None, np.zeros((5, 2)), np.zeros((5, 2)), np.eye(3))
    with pytest.raises(cv.error):
        cv.xfeatures2d.SIFT_create(nOctaveLayers=4)  # only SIFT_create()'s defaults (v3:100)
    with pytest.raises(cv.error):
        cv.xfeatures2d.SURF_create(400, extended=True)  # only SURF_create(400)'s other defaults (v3:104)
    with pytest.raises(cv.error):
        cv.xfeatures2d.SURF_create(400).detectAndCompute(np.zeros((8, 8), np.uint8), np.ones((8, 8), np.uint8))
    with pytest.raises(cv.error):
        cv.SIFT_create().detectAndCompute(np.zeros((8, 8), np.uint8), np.ones((8, 8), np.uint8))
    with pytest.raises(cv.error):
        cv.BFMatcher(cv.NORM_HAMMING, True).knnMatch(None, None, k=2)
    with pytest.raises(cv.error):
        cv.triangulatePoints(None, np.zeros((3, 4)), np.zeros((2, 1)), np.zeros((2, 1)))


@pytest.mark.parametrize("dist,size", [
    (np.zeros(5), (640, 480)),
    (np.array([0.142541, -0.248887, -0.005254, -0.005417, 0.0]), (640, 480)),      # rosbot_calibration.yaml:22
    (np.array([-0.296079, 0.099771, 0.000222, 0.000109, 0.0]), (1440, 1080)),      # camera_calibration.yaml:22
    (np.array([0.1, -0.2, 0.001, -0.002, 0.05, 0.01, -0.02, 0.003]), (1280, 720)),  # rational model
])
def test_optimal_new_camera_matrix_matches_oracle(oracle_mod, dist, size):
    """Host arithmetic of cv.getOptimalNewCameraMatrix(K, dist, size, 1, size)
    (v3:117) in the library == the oracle restatement, bit for bit."""
    K = np.array([[606.811009, 0, 325.199941], [0, 611.104701, 227.591593], [0, 0, 1.0]])
    if size[0] > 640:
        K = np.array([[1173.854081, 0, 747.788206], [0, 1170.565083, 574.700374], [0, 0, 1.0]])
    got, roi = cv.getOptimalNewCameraMatrix(K, dist, size, 1, size)
    want = oracle_mod.get_optimal_new_camera_matrix(K, dist, size[0], size[1], 1.0)
    np.testing.assert_array_equal(got, want)
    assert roi == (0, 0, size[0], size[1])
    if not np.any(dist):
        # zero distortion: K scaled by (w-1)/w, (h-1)/h (the inner rectangle is the image)
        np.testing.assert_allclose(got[0, 0], K[0, 0] * (size[0] - 1) / size[0], rtol=1e-6)


def test_bad_distortion_length_raises():
    with pytest.raises(cv.error):
        cv.getOptimalNewCameraMatrix(np.eye(3), np.zeros(3), (64, 48), 1, (64, 48))


def test_imdecode_png_round_trip(tmp_path):
    img = (np.arange(48 * 3).reshape(4, 12, 3) * 5 % 256).astype(np.uint8)
    p = tmp_path / "a.png"
    cv.imwrite(str(p), img)
    back = cv.imdecode(np.frombuffer(p.read_bytes(), np.uint8), cv.IMREAD_COLOR)
    np.testing.assert_array_equal(back, img)
    assert cv.imdecode(np.zeros(10, np.uint8)) is None


def test_draw_keypoints_circle():
    img = np.zeros((20, 20), np.uint8)
    out = cv.drawKeypoints(img, [cv.KeyPoint(10, 10, 31)], None, color=(0, 255, 0))
    assert out.shape == (20, 20, 3)
    assert tuple(out[10, 13]) == (0, 255, 0) and tuple(out[10, 10]) == (0, 0, 0)


CONTROLLED_YAML = """camera_matrix:
  rows: 3
  cols: 3
  data: [500.0, 0.0, 320.0, 0.0, 500.0, 240.0, 0.0, 0.0, 1.0]
distortion_coefficients:
  rows: 1
  cols: 5
  data: [0.0, 0.0, 0.0, 0.0, 0.0]
"""


@pytest.fixture
def vo_module():
    sys.path.insert(0, os.path.join(ROOT, "droplet_visual_odometry_amd", "dropin"))
    try:
        import visual_odometry_v3
        yield visual_odometry_v3
    finally:
        sys.path.pop(0)


def test_dropin_constructs_and_parses_yaml(vo_module, tmp_path):
    y = tmp_path / "cal.yaml"
    y.write_text(CONTROLLED_YAML)
    vo = vo_module.VisualOdometry(to_sort=True, mode="orb", calibration_file_path=str(y), controlled=True,
                                  real_marker_length=0.1)
    np.testing.assert_array_equal(vo.intrinsic_coefficient_matrix, [[500, 0, 320], [0, 500, 240], [0, 0, 1]])
    assert vo.distortion_coefficient_matrix.shape == (1, 5)
    np.testing.assert_array_equal(vo.previous_projection_matrix, np.hstack((vo.intrinsic_coefficient_matrix,
                                                                            np.zeros((3, 1)))))
    assert (vo.frame_width, vo.frame_height) == (640, 480)
    assert vo.norm_type == cv.NORM_HAMMING and vo.cross_check is True
    np.testing.assert_array_equal(vo.robot_curr_position, np.eye(4))
    assert vo_module.number_of_frames == 25075


def test_dropin_non_controlled_reference_yaml(vo_module, tmp_path):
    y = tmp_path / "cal.yaml"
    y.write_text("distortion_coeffs:\n- [0.1, -0.2, 0.0, 0.0, 0.0]\nintrinsic_coeffs:\n"
                 "- [606.8, 0.0, 325.2, 0.0, 611.1, 227.6, 0.0, 0.0, 1.0]\n")
    vo = vo_module.VisualOdometry(mode="orb", calibration_file_path=str(y), controlled=False)
    assert vo.previous_projection_matrix is None           # D2
    assert vo.intrinsic_coefficient_matrix[0, 0] == 606.8
    assert (vo.frame_width, vo.frame_height) == (1400, 1080)


def test_dropin_unknown_message_type(vo_module, tmp_path):
    y = tmp_path / "cal.yaml"
    y.write_text(CONTROLLED_YAML)
    vo = vo_module.VisualOdometry(mode="orb", calibration_file_path=str(y), controlled=True)
    msg = types.SimpleNamespace(data=b"", height=480, width=640)
    with pytest.raises(cv.error):  # image_np stays None, cvtColor asserts in the reference
        vo.ros_img_msg_to_opencv_image(msg, "unknown")


def test_dropin_make_transform_mat(vo_module, tmp_path):
    from droplet_visual_odometry_amd import transformations as tr
    y = tmp_path / "cal.yaml"
    y.write_text(CONTROLLED_YAML)
    vo = vo_module.VisualOdometry(mode="orb", calibration_file_path=str(y), controlled=True)
    T = vo.make_transform_mat([1, 2, 3], [0.1, 0.2, 0.3])
    np.testing.assert_allclose(T[:3, :3], tr.euler_matrix(0.1, 0.2, 0.3, "sxyz")[:3, :3])
    np.testing.assert_array_equal(T[:3, 3], [1, 2, 3])


def test_feature_cache_lru(vo_module):
    c = vo_module._FeatureCache(size=2)
    a, b, d = (np.full((2, 2), v, np.uint8) for v in (1, 2, 3))
    for x in (a, b):
        c.put(c.key(x), x)
    assert c.get(c.key(a)) is a
    c.put(c.key(d), d)                                      # evicts b (least recent)
    assert c.get(c.key(b)) is None and c.get(c.key(a)) is a
    assert c.key(a) != c.key(a.astype(np.uint16))
