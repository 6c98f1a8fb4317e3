"""Drop-in replacement for the reference's scripts/visual_odometry_v3.py.

Put this directory (droplet_visual_odometry_amd/dropin) first on sys.path and
`from visual_odometry_v3 import VisualOdometry` (trajectory_evaluation_dual_process.py:21)
gets this class: same constructor, methods, attributes and module constants,
with every OpenCV operator on the hot path served by the MI355X kernels through
droplet_visual_odometry_amd.cv.

Behaviour notes versus the reference:
  D1  the ORB branch of get_matches_between_two_frames indexes `m[0]` on plain
      DMatch objects (v3:233-238) and raises TypeError under cv2; our DMatch
      supports `m[0] is m`, so the loop runs as the author intended.
  D2  non-controlled calibration leaves previous_projection_matrix None and the
      first triangulation fails exactly as in the reference (cv.error).
  D3  the scale uses the raw homogeneous X, Y, Z of the triangulated corners.
  D4  Euler angles are extracted with 'rxyz' and rebuilt with 'sxyz'.
  D5  both frames are detected every call, as in the reference; a
      content-keyed cache (identical outputs) skips re-detecting the previous
      frame when the same bytes come back.
  D6  drawKeypoints is returned lazily: the drawn image is made the first
      time a caller reads it (the reference computes it and discards it).
  D7  fused pair path: with the stock ORB / BFMatcher(NORM_HAMMING, crossCheck)
      operators (mode "orb", no method overridden), visual_odometry_calculations
      runs detect -> match -> findEssentialMat -> recoverPose in ONE library
      call (FrameStream.pair / dvo_stream_pair; the previous frame's features
      stay on the device when its bytes come back as the next previous frame),
      then the same host tail (triangulation, scale, Euler rebuild) as the
      operator-by-operator path, so the 4x4s are identical.  Any pair the
      library reports as failing (status, or not exactly one E) is redone
      operator by operator, which raises where the reference raises.

Matches and keypoints are array-backed sequences (cv.DMatches, cv.KeyPoints):
the ORB branch sorts by distance with a stable argsort (Python's sorted() is
stable, v3:221) and gathers the matched keypoints by index, instead of
building and walking thousands of Python objects per pair.
"""
from __future__ import annotations

import hashlib
import logging
import math
from collections import OrderedDict

import numpy as np
import yaml
from yaml.loader import SafeLoader

from droplet_visual_odometry_amd import cv
from droplet_visual_odometry_amd import transformations as transf

log = logging.getLogger("visual_odometry_v3")

VERBOSE = False
number_of_frames = 25075
DEFAULT_STARTING_ROBOT_TRANSLATION = [0, 0, 0]
DEFAULT_STARTING_ROBOT_EULER = [0, 0, 0]


try:  # 128-bit content hash: xxh3 (~20 GB/s) when installed, else blake2b
    import xxhash

    def _digest(buf):
        return xxhash.xxh3_128_digest(buf)
except ImportError:  # pragma: no cover
    def _digest(buf):
        return hashlib.blake2b(buf, digest_size=16).digest()


class _LazyDrawing:
    """cv.drawKeypoints(image, kps, None, color=(0, 255, 0), flags=0) made on
    first use: behaves as the drawn uint8[H, W, 3] image."""

    def __init__(self, image, kps):
        self._args = (image, kps)
        self._img = None

    def _get(self):
        if self._img is None:
            image, kps = self._args
            self._img = cv.drawKeypoints(image, kps, None, color=(0, 255, 0), flags=0)
        return self._img

    def __array__(self, dtype=None, copy=None):
        a = self._get()
        return a if dtype is None else a.astype(dtype)

    def __getattr__(self, name):
        return getattr(self._get(), name)

    def __getitem__(self, i):
        return self._get()[i]

    def __len__(self):
        return len(self._get())


class _FeatureCache:
    """Content-keyed LRU of (keypoints, descriptors, drawn image)."""

    def __init__(self, size=4):
        self.size = size
        self.d = OrderedDict()

    @staticmethod
    def key(img):
        a = np.ascontiguousarray(img)
        return (a.shape, a.dtype.str, _digest(a.data))

    def get(self, k):
        v = self.d.get(k)
        if v is not None:
            self.d.move_to_end(k)
        return v

    def put(self, k, v):
        self.d[k] = v
        self.d.move_to_end(k)
        while len(self.d) > self.size:
            self.d.popitem(last=False)


class VisualOdometry:
    """Per-frame-pair visual odometry (visual_odometry_v3.py:26-408)."""

    def __init__(self, starting_translation=None, starting_euler=None, to_sort=False, mode="ORB",
                 calibration_file_path="", controlled=False, real_marker_length=0.0):
        self.starting_euler = DEFAULT_STARTING_ROBOT_EULER if starting_euler is None else starting_euler
        self.starting_translation = (DEFAULT_STARTING_ROBOT_TRANSLATION if starting_translation is None
                                     else starting_translation)
        self.controlled = controlled
        # v3:39-44: usb_cam frames are 640x480, compressed camera_array frames 1400x1080
        self.frame_width, self.frame_height = (640, 480) if controlled else (1400, 1080)
        log.debug("controlled=%s frame %dx%d", controlled, self.frame_width, self.frame_height)

        self.robot_current_translation = None
        self.essential_matrix = None
        self.calibration_file_path = calibration_file_path
        self.distortion_coefficient_matrix = None
        self.intrinsic_coefficient_matrix = None
        self.previous_projection_matrix = None
        self.parse_camera_intrinsics()

        self.to_sort = to_sort
        self.mode = mode
        self.real_marker_length = real_marker_length
        self.feature_detector, self.norm_type, self.cross_check = self.return_feature_matching_parameters(mode)
        self.bf = cv.BFMatcher(normType=self.norm_type, crossCheck=self.cross_check)

        self.robot_position_list = []
        self.ground_truth_list = []
        self.frame_translations = []
        self.matches_dictionary = []
        self.projection_matrix_list = []
        self.plot_4D_counter = 1
        self._features = _FeatureCache()
        self._pair_engine = None  # (config key, FrameStream) of the fused pair path (D7)
        self._pair_last = None    # content key of the last fused pair's current frame
        self.robot_curr_position = self.make_transform_mat(translation=self.starting_translation,
                                                           euler=self.starting_euler)

    # ---- utilities (v3:93-167) -------------------------------------------------
    def return_feature_matching_parameters(self, mode):
        """(detector, normType, crossCheck) for the matching mode (v3:93-107)."""
        global feature_detector, norm_type, cross_check
        m = mode.lower()
        if m == "orb":
            feature_detector, norm_type, cross_check = cv.ORB_create(), cv.NORM_HAMMING, True
        elif m in ("sift", "flann", "knn_sift"):
            feature_detector, norm_type, cross_check = cv.xfeatures2d.SIFT_create(), cv.NORM_L1, False
        elif m == "surf":
            feature_detector, norm_type, cross_check = cv.xfeatures2d.SURF_create(400), cv.NORM_L1, False
        return feature_detector, norm_type, cross_check

    def undistort_image(self, distorted_image, new_camera_matrix):
        return cv.undistort(src=distorted_image, cameraMatrix=self.intrinsic_coefficient_matrix,
                            distCoeffs=self.distortion_coefficient_matrix, newCameraMatrix=new_camera_matrix)

    def ros_img_msg_to_opencv_image(self, image_message, msg_type):
        """ROS image message -> undistorted mono8 (v3:115-135)."""
        size = (self.frame_width, self.frame_height)
        new_camera_matrix, _ = cv.getOptimalNewCameraMatrix(self.intrinsic_coefficient_matrix,
                                                            self.distortion_coefficient_matrix, size, 1, size)
        image_np = None
        if msg_type == "compressed":
            image_np = cv.imdecode(np.frombuffer(image_message.data, np.uint8), cv.IMREAD_COLOR)
        elif msg_type == "usb_raw":
            raw = np.frombuffer(image_message.data, dtype=np.uint8)
            image_np = raw.reshape((image_message.height, image_message.width, -1))
        if image_np is None:
            raise cv.error("(-215:Assertion failed) !_src.empty() in function 'cvtColor'")
        grey_image = cv.cvtColor(src=image_np, code=cv.COLOR_BGR2GRAY)
        return self.undistort_image(grey_image, new_camera_matrix)

    def make_transform_mat(self, translation, euler):
        """translation_matrix(t) . euler_matrix(rx, ry, rz, 'sxyz') (v3:138-142)."""
        rx, ry, rz = euler
        rotation = transf.euler_matrix(rx, ry, rz, axes="sxyz")
        return transf.translation_matrix(translation).dot(rotation)

    def parse_camera_intrinsics(self):
        """K and distortion from the calibration YAML (v3:145-167)."""
        with open(self.calibration_file_path) as fh:
            data = yaml.load(fh, Loader=SafeLoader)
        if not self.controlled:
            self.distortion_coefficient_matrix = np.array(data["distortion_coeffs"][0])
            self.intrinsic_coefficient_matrix = np.array(data["intrinsic_coeffs"][0]).reshape((3, 3))
        else:
            self.intrinsic_coefficient_matrix = np.array(data["camera_matrix"]["data"]).reshape((3, 3))
            self.distortion_coefficient_matrix = np.array(data["distortion_coefficients"]["data"]).reshape((1, 5))
            self.previous_projection_matrix = np.matmul(self.intrinsic_coefficient_matrix,
                                                        np.hstack((np.eye(3), np.zeros((3, 1)))))

    # ---- the per-pair path (v3:191-408) ----------------------------------------
    def visualize_key_points_matching(self, *args, **kwargs):
        raise cv.error("visualisation (drawMatches/imshow, v3:172-189) is out of scope")

    def get_matches_between_two_frames(self, previous_key_points, previous_descriptors, current_key_points,
                                       current_descriptors):
        """Match previous (query) to current (train) descriptors (v3:191-239)."""
        matches = None
        if self.mode == "sift":
            matches = self.bf.match(previous_descriptors, current_descriptors)
        elif self.mode in ("knn_sift", "surf"):
            matches = self.bf.knnMatch(previous_descriptors, current_descriptors, k=2)
        elif self.mode == "flann":
            flann = cv.FlannBasedMatcher(dict(algorithm=1, trees=5), dict(checks=50))
            matches = flann.knnMatch(previous_descriptors, current_descriptors, k=2)
        elif self.mode == "orb":
            matches = self.bf.match(previous_descriptors, current_descriptors)
            if isinstance(matches, cv.DMatches):
                matches = matches.sorted_by_distance()
                if isinstance(previous_key_points, cv.KeyPoints) and isinstance(current_key_points, cv.KeyPoints):
                    return (matches, previous_key_points.take(matches.array["queryIdx"]),
                            current_key_points.take(matches.array["trainIdx"]))
            else:
                matches = sorted(matches, key=lambda x: x.distance)
        if self.mode != "orb":
            passed = [[m] for m, n in matches if m.distance < 0.75 * n.distance]
        else:
            passed = matches
        top_prev, top_cur = [], []
        for entry in passed:
            m = entry[0]
            top_prev.append(previous_key_points[m.queryIdx])
            top_cur.append(current_key_points[m.trainIdx])
        return matches, top_prev, top_cur

    def visualize_4D_marker_corners(self, marker_corners_4D, path=None):
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        fig = plt.figure()
        ax = fig.add_subplot(111, projection="3d")
        ax.scatter(marker_corners_4D[0, :], marker_corners_4D[1, :], marker_corners_4D[2, :])
        ax.set_xlabel("marker_corners_X")
        ax.set_ylabel("marker_corners_Y")
        ax.set_zlabel("marker_corners_Z")
        if path:
            fig.savefig(path)
        plt.close(fig)
        self.plot_4D_counter += 1

    def get_scaling_factor_from_triangulation(self, current_projection_matrix, previous_marker_corners,
                                              current_marker_corners):
        """Distance between the first two triangulated marker corners (v3:263-291).

        The corners are not dehomogenised (D3); the caller divides the real
        marker length by the returned distance."""
        self.projection_matrix_list.append(self.previous_projection_matrix)
        X = cv.triangulatePoints(projMatr1=self.previous_projection_matrix, projMatr2=current_projection_matrix,
                                 projPoints1=previous_marker_corners.T, projPoints2=current_marker_corners.T)
        dx, dy, dz = X[0, 0] - X[0, 1], X[1, 0] - X[1, 1], X[2, 0] - X[2, 1]
        real_world_distance = math.sqrt(dx ** 2 + dy ** 2 + dz ** 2)
        log.debug("marker corner distance %s (real length %s)", real_world_distance, self.real_marker_length)
        return real_world_distance

    def get_transformation_between_two_frames(self, array_previous_key_points, array_current_key_points,
                                              previous_marker_corners, current_marker_corners):
        """E (RANSAC) -> R, t -> marker scale -> 4x4 previous->current (v3:293-345)."""
        K = self.intrinsic_coefficient_matrix
        self.essential_matrix, _mask = cv.findEssentialMat(points1=array_previous_key_points,
                                                           points2=array_current_key_points, cameraMatrix=K,
                                                           method=cv.RANSAC, prob=0.999, threshold=1.0)
        _good, relative_rotation, translation, _mask = cv.recoverPose(E=self.essential_matrix,
                                                                      points1=array_previous_key_points,
                                                                      points2=array_current_key_points,
                                                                      cameraMatrix=K)
        return self._relative_transform(relative_rotation, translation, previous_marker_corners,
                                        current_marker_corners)

    def _relative_transform(self, relative_rotation, translation, previous_marker_corners, current_marker_corners):
        """v3:305-345: P_cur = K [R | t], marker scale, 4x4 previous->current."""
        K = self.intrinsic_coefficient_matrix
        current_projection_matrix = K.dot(np.hstack((relative_rotation, translation.reshape(-1, 1))))
        distance = self.get_scaling_factor_from_triangulation(current_projection_matrix=current_projection_matrix,
                                                              previous_marker_corners=previous_marker_corners,
                                                              current_marker_corners=current_marker_corners)
        scaling_factor = self.real_marker_length / distance
        translation = translation.transpose()[0] * scaling_factor
        rotation4 = np.vstack((np.hstack((np.array(relative_rotation), np.array([0, 0, 0])[:, None])), [0, 0, 0, 1]))
        euler = np.array(transf.euler_from_matrix(rotation4, "rxyz"))
        prev_to_curr = self.make_transform_mat(translation=translation, euler=euler)
        self.frame_translations.append(prev_to_curr)
        self.previous_projection_matrix = current_projection_matrix
        return prev_to_curr

    def previous_current_matching(self, top_previous_key_points, top_current_key_points,
                                  robot_previous_position_transformation, previous_marker_corners,
                                  current_marker_corners):
        """KeyPoint_convert, relative transform, T_robot_cur = T_robot_prev . T (v3:349-368)."""
        p_prev = cv.KeyPoint_convert(top_previous_key_points)
        p_cur = cv.KeyPoint_convert(top_current_key_points)
        rel = self.get_transformation_between_two_frames(p_prev, p_cur, previous_marker_corners,
                                                         current_marker_corners)
        return robot_previous_position_transformation.dot(rel), rel

    def compute_current_image_elements(self, input_image):
        """ORB keypoints, descriptors and the drawn keypoint image (v3:370-379)."""
        key = _FeatureCache.key(input_image)
        hit = self._features.get(key)
        if hit is None:
            kps, desc = self.feature_detector.detectAndCompute(input_image, None)
            hit = (kps, desc, _LazyDrawing(np.array(input_image, copy=True), kps))
            self._features.put(key, hit)
        return hit

    def _fused_pair(self, previous_image, current_image):
        """(E, R, t) of the pair from one library call (D7), or None when the
        stock operators are not in use or the library reports a failing pair."""
        cls = type(self)
        if (self.mode != "orb" or type(self.feature_detector) is not cv.ORB or type(self.bf) is not cv.BFMatcher
                or self.bf.normType != cv.NORM_HAMMING or not self.bf.crossCheck
                or any(getattr(cls, m) is not getattr(VisualOdometry, m) for m in (
                    "compute_current_image_elements", "get_matches_between_two_frames", "previous_current_matching",
                    "get_transformation_between_two_frames"))):
            return None
        prev = np.asarray(previous_image)
        cur = np.asarray(current_image)
        if prev.dtype != np.uint8 or cur.dtype != np.uint8 or prev.ndim != 2 or prev.shape != cur.shape:
            return None
        h, w = cur.shape
        if not (8 <= w < 4096 and 8 <= h < 4096):
            return None
        K = np.ascontiguousarray(self.intrinsic_coefficient_matrix, np.float64)
        if K.shape != (3, 3):
            return None
        det = self.feature_detector
        cc = 2 if self.bf.legacy_crosscheck else 1
        cfg = (w, h, det.nfeatures, det.fastThreshold, det.opencv, K.tobytes(), cc)
        if self._pair_engine is None or self._pair_engine[0] != cfg:
            from droplet_visual_odometry_amd import ops
            self._pair_engine = None
            self._pair_last = None
            self._pair_engine = (cfg, ops.PairStream(w, h, K, nfeatures=det.nfeatures, fast_threshold=det.fastThreshold,
                                                     cross_check=cc, opencv=det.opencv))
        fs = self._pair_engine[1]
        kprev, kcur = _FeatureCache.key(prev), _FeatureCache.key(cur)
        reuse = self._pair_last is not None and self._pair_last == kprev
        self._pair_last = None
        rec = fs.pair(None if reuse else prev, cur, reuse_prev=reuse)
        self._pair_last = kcur
        if rec["status"] != 0 or rec["n_models"] != 1:
            return None
        return rec["E"].reshape(3, 3).copy(), rec["R"].reshape(3, 3).copy(), rec["t"].reshape(3, 1).copy()

    def visual_odometry_calculations(self, previous_image, current_image, robot_previous_position_transformation,
                                     previous_marker_corners, current_marker_corners):
        """(T_robot_current, T_previous_to_current) for one frame pair (v3:384-408)."""
        fused = self._fused_pair(previous_image, current_image)
        if fused is not None:  # D7: detect -> match -> E -> R, t in one call, then the same host tail
            self.essential_matrix, relative_rotation, translation = fused
            rel = self._relative_transform(relative_rotation, translation, previous_marker_corners,
                                           current_marker_corners)
            return robot_previous_position_transformation.dot(rel), rel
        prev_kp, prev_desc, _ = self.compute_current_image_elements(previous_image)
        cur_kp, cur_desc, _ = self.compute_current_image_elements(current_image)
        _matches, top_prev, top_cur = self.get_matches_between_two_frames(
            previous_key_points=prev_kp, previous_descriptors=prev_desc,
            current_key_points=cur_kp, current_descriptors=cur_desc)
        return self.previous_current_matching(top_prev, top_cur, robot_previous_position_transformation,
                                              previous_marker_corners, current_marker_corners)


if __name__ == "__main__":
    pass
