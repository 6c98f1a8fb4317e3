"""The slice of the `cv2` API the reference's hot path uses, backed by the MI355X kernels.

The reference calls (scripts/visual_odometry_v3.py):
  cv.ORB_create()                                       :96
  cv.BFMatcher(normType=NORM_HAMMING, crossCheck=True)  :75    .match :219
  cv.BFMatcher(normType=NORM_L1) .match / .knnMatch(k=2) :99-106, :200-204, :214-215 (SIFT/SURF)
  cv.FlannBasedMatcher(index, search).knnMatch(k=2)     :206-212 (exact-search stand-in)
  cv.xfeatures2d.SIFT_create()                          :100 (GPU; SURF_create(400), :104, host cv2 contrib only)
  detector.detectAndCompute(img, None)                  :373
  cv.drawKeypoints(img, kps, None, color, flags=0)      :375   (result discarded, D6)
  cv.KeyPoint_convert(kps)                              :355, :358
  cv.findEssentialMat(points1=, points2=, cameraMatrix=, method=RANSAC, prob=, threshold=)   :297
  cv.recoverPose(E=, points1=, points2=, cameraMatrix=) :303
  cv.triangulatePoints(projMatr1=, projMatr2=, projPoints1=, projPoints2=)                 :265
These keep OpenCV's Python signatures, return types and failure points
(`cv.error` where cv2 raises cv2.error).  Pre-processing helpers used by
ros_img_msg_to_opencv_image (imdecode, cvtColor, undistort,
getOptimalNewCameraMatrix; v3:110-135) are outside the GPU hot path (SURVEY.md
§8f, "next") and are implemented on the host with the restrictions documented
on each.
"""
from __future__ import annotations

import os
from collections.abc import Sequence

import numpy as np

from . import ops
from ._native import DVOError, opencv_semantics

# Which OpenCV release's semantics the cv2 stand-ins reproduce (include/dvo.h
# DVO_OPENCV_*): "4.x" by default, or "3.2" -- the version the reference most
# likely ran (ROS Melodic, Python 2.7): ORB's INTER_LINEAR
# pyramid and retainBest, and BFMatcher's 3.x cross check.  Set
# DVO_OPENCV_SEMANTICS=3.2 in the environment (read at import), or assign
# cv.OPENCV_SEMANTICS before creating the detector / matcher.
OPENCV_SEMANTICS = os.environ.get("DVO_OPENCV_SEMANTICS", "4.x")
opencv_semantics(OPENCV_SEMANTICS)  # validate

# cv2 constants used by the reference
NORM_L1 = 2
NORM_L2 = 4
NORM_HAMMING = 6
NORM_HAMMING2 = 7
RANSAC = 8
LMEDS = 4
IMREAD_COLOR = 1
IMREAD_GRAYSCALE = 0
COLOR_BGR2GRAY = 6
COLOR_GRAY2BGR = 8
DrawMatchesFlags_DEFAULT = 0
DrawMatchesFlags_NOT_DRAW_SINGLE_POINTS = 2


class error(Exception):
    """cv2.error analogue."""


class KeyPoint:
    """cv2.KeyPoint (pt, size, angle, response, octave, class_id)."""
    __slots__ = ("pt", "size", "angle", "response", "octave", "class_id")

    def __init__(self, x=0.0, y=0.0, size=0.0, angle=-1.0, response=0.0, octave=0, class_id=-1):
        self.pt = (float(x), float(y))
        self.size = float(size)
        self.angle = float(angle)
        self.response = float(response)
        self.octave = int(octave)
        self.class_id = int(class_id)

    def __repr__(self):
        return f"<KeyPoint pt={self.pt} size={self.size} angle={self.angle} response={self.response} octave={self.octave}>"


class DMatch:
    """cv2.DMatch.  `m[0]` returns `m` itself so the reference's ORB loop
    (v3:233-238, written for k-NN match lists) runs unchanged."""
    __slots__ = ("queryIdx", "trainIdx", "imgIdx", "distance")

    def __init__(self, queryIdx=-1, trainIdx=-1, imgIdx=0, distance=float("inf")):
        self.queryIdx = int(queryIdx)
        self.trainIdx = int(trainIdx)
        self.imgIdx = int(imgIdx)
        self.distance = float(distance)

    def __getitem__(self, i):
        if i == 0 or i == -1:
            return self
        raise IndexError("DMatch index out of range")

    def __repr__(self):
        return f"<DMatch q={self.queryIdx} t={self.trainIdx} d={self.distance}>"


class KeyPoints(Sequence):
    """The keypoint sequence detectAndCompute returns (cv2 returns a tuple of
    KeyPoint), backed by the structured array the library wrote
    (KEYPOINT_DTYPE).  KeyPoint objects are built on first access, so a frame's
    2000 keypoints cost no Python objects until someone indexes them;
    KeyPoint_convert and the drop-in's match gather work on the array."""
    __slots__ = ("array", "_objs")

    def __init__(self, array: np.ndarray):
        self.array = array
        self._objs = None

    def __len__(self):
        return len(self.array)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return KeyPoints(self.array[i])
        n = len(self.array)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError("keypoint index out of range")
        if self._objs is None:
            self._objs = [None] * n
        k = self._objs[i]
        if k is None:
            k = self._objs[i] = KeyPoint(*self.array[i].tolist())
        return k

    def take(self, idx) -> "KeyPoints":
        """Keypoints at the given indices (a gather on the array)."""
        return KeyPoints(self.array[np.asarray(idx, np.int64)])

    def __add__(self, other):
        return tuple(self) + tuple(other)

    def __repr__(self):
        return f"<KeyPoints n={len(self)}>"


class DMatches(Sequence):
    """The match sequence BFMatcher.match returns, backed by a DMATCH_DTYPE
    array; DMatch objects are built on first access."""
    __slots__ = ("array", "_objs")

    def __init__(self, array: np.ndarray):
        self.array = array
        self._objs = None

    def __len__(self):
        return len(self.array)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return DMatches(self.array[i])
        n = len(self.array)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError("match index out of range")
        if self._objs is None:
            self._objs = [None] * n
        m = self._objs[i]
        if m is None:
            r = self.array[i]
            m = self._objs[i] = DMatch(int(r["queryIdx"]), int(r["trainIdx"]), int(r["imgIdx"]), float(r["distance"]))
        return m

    def sorted_by_distance(self) -> "DMatches":
        """sorted(matches, key=lambda m: m.distance) (visual_odometry_v3.py:221):
        Python's sort is stable, so is this argsort."""
        return DMatches(self.array[np.argsort(self.array["distance"], kind="stable")])

    def __add__(self, other):
        return list(self) + list(other)

    def __repr__(self):
        return f"<DMatches n={len(self)}>"


def KeyPoint_convert(keypoints, keypointIndexes=None):
    """float32[N, 2] of keypoint coordinates (cv2.KeyPoint_convert)."""
    if isinstance(keypoints, KeyPoints):
        arr = keypoints.array if keypointIndexes is None else keypoints.array[np.asarray(keypointIndexes, np.int64)]
        return np.stack([arr["x"], arr["y"]], axis=1).astype(np.float32)
    kps = keypoints if keypointIndexes is None else [keypoints[i] for i in keypointIndexes]
    if len(kps) == 0:
        return np.zeros((0, 2), np.float32)
    return np.array([k.pt for k in kps], dtype=np.float32)


class ORB:
    """cv2.ORB with the ORB_create() defaults (v3:96); nfeatures configurable."""

    def __init__(self, nfeatures=500, scaleFactor=1.2, nlevels=8, edgeThreshold=31, firstLevel=0, WTA_K=2,
                 scoreType=0, patchSize=31, fastThreshold=20):
        if (np.float32(scaleFactor) != np.float32(1.2) or nlevels != 8 or edgeThreshold != 31 or firstLevel != 0
                or WTA_K != 2 or scoreType != 0 or patchSize != 31):
            raise error("only the cv.ORB_create() defaults (other than nfeatures/fastThreshold) are implemented")
        self.nfeatures = int(nfeatures)
        self.fastThreshold = int(fastThreshold)
        self.opencv = OPENCV_SEMANTICS

    def getMaxFeatures(self):
        return self.nfeatures

    def setMaxFeatures(self, n):
        self.nfeatures = int(n)

    def detectAndCompute(self, image, mask, descriptors=None, useProvidedKeypoints=False):
        if mask is not None:
            raise error("ORB masks are not supported (the reference passes None, v3:373)")
        if useProvidedKeypoints:
            raise error("useProvidedKeypoints is not supported")
        img = _gray(image)
        try:
            kps, desc = ops.detect_and_compute(img, self.nfeatures, self.fastThreshold, self.opencv)
        except DVOError as e:
            raise error(str(e)) from e
        return KeyPoints(kps), (desc if len(kps) else None)

    def detect(self, image, mask=None):
        return self.detectAndCompute(image, mask)[0]


def ORB_create(nfeatures=500, scaleFactor=1.2, nlevels=8, edgeThreshold=31, firstLevel=0, WTA_K=2, scoreType=0,
               patchSize=31, fastThreshold=20):
    return ORB(nfeatures, scaleFactor, nlevels, edgeThreshold, firstLevel, WTA_K, scoreType, patchSize, fastThreshold)


def _float_desc(d):
    a = np.asarray(d)
    if a.ndim != 2 or a.dtype != np.float32:
        raise error("(-215:Assertion failed) NORM_L1 / FLANN matching needs float32 [N, dim] descriptors")
    return a


def _knn_lists(q, t, k, norm, sqrt_dist=False):
    if len(q) == 0 or len(t) == 0:
        return [[] for _ in range(len(q))] if len(t) == 0 else []
    if q.shape[1] != t.shape[1]:
        raise error("(-215:Assertion failed) query and train descriptors differ in length")
    try:
        idx, dist = ops.bf_knn_float(q, t, k, norm)
    except DVOError as e:
        raise error(str(e)) from e
    if sqrt_dist:
        # FlannBasedMatcher::convertToDMatches: float FLANN distances (squared L2)
        # become std::sqrt(float) in DMatch.distance; ranking stays on the squares
        dist = np.sqrt(dist.astype(np.float32))
    out = []
    for qi in range(len(q)):
        row = []
        for s in range(k):
            if idx[qi, s] < 0:
                break
            row.append(DMatch(qi, int(idx[qi, s]), 0, float(dist[qi, s])))
        out.append(row)
    return out


class BFMatcher:
    """cv2.BFMatcher: NORM_HAMMING (the ORB branch, v3:75, v3:97) and NORM_L1
    on float descriptors (the SIFT/SURF branches, v3:99-106).

    crossCheck follows OpenCV 4.x (mutual nearest neighbour) unless
    legacy_crosscheck=True (default: OPENCV_SEMANTICS == "3.2") selects OpenCV
    3.x's reverse-pass semantics; it is implemented for NORM_HAMMING (the
    reference sets it only there)."""

    def __init__(self, normType=NORM_L2, crossCheck=False, legacy_crosscheck=None):
        self.normType = normType
        self.crossCheck = bool(crossCheck)
        self.legacy_crosscheck = (opencv_semantics(OPENCV_SEMANTICS) == 1 if legacy_crosscheck is None
                                  else bool(legacy_crosscheck))

    def _check_l1(self):
        if self.normType != NORM_L1:
            raise error("only NORM_HAMMING (ORB) and NORM_L1 (SIFT/SURF) are implemented on the GPU")
        if self.crossCheck:
            raise error("crossCheck is implemented for NORM_HAMMING only (the reference's L1 modes pass False)")

    def match(self, queryDescriptors, trainDescriptors, mask=None):
        if mask is not None:
            raise error("match masks are not supported")
        if queryDescriptors is None or trainDescriptors is None:
            raise error("(-215:Assertion failed) descriptors must not be empty")
        if self.normType != NORM_HAMMING:
            self._check_l1()
            return [row[0] for row in _knn_lists(_float_desc(queryDescriptors), _float_desc(trainDescriptors), 1,
                                                 ops.NORM_L1) if row]
        q = np.asarray(queryDescriptors)
        t = np.asarray(trainDescriptors)
        if q.dtype != np.uint8 or t.dtype != np.uint8 or q.shape[-1] != 32 or t.shape[-1] != 32:
            raise error("(-215:Assertion failed) NORM_HAMMING needs uint8 descriptors of 32 bytes")
        mode = 0 if not self.crossCheck else (2 if self.legacy_crosscheck else 1)
        try:
            m = ops.bf_match(q, t, mode)
        except DVOError as e:
            raise error(str(e)) from e
        return DMatches(m)

    def knnMatch(self, queryDescriptors, trainDescriptors, k, mask=None, compactResult=False):
        """List (one per query) of up to k DMatch in ascending distance."""
        if mask is not None:
            raise error("match masks are not supported")
        if queryDescriptors is None or trainDescriptors is None:
            raise error("(-215:Assertion failed) descriptors must not be empty")
        self._check_l1()
        out = _knn_lists(_float_desc(queryDescriptors), _float_desc(trainDescriptors), int(k), ops.NORM_L1)
        return [r for r in out if r] if compactResult else out


# cv::theRNG(): per-thread process state in OpenCV.  FLANN's kd-tree builds draw
# from it (every FlannBasedMatcher.knnMatch builds an index), so the stand-in
# carries it across calls the same way (cv2.setRNGSeed resets it).
import threading as _threading

_rng_tls = _threading.local()


def _the_rng():
    st = getattr(_rng_tls, "state", None)
    return ops.THE_RNG_SEED if st is None else st


def setRNGSeed(seed):
    """cv2.setRNGSeed(int): theRNG() = RNG((uint64)seed); RNG(0) starts at 0xFFFFFFFF."""
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    _rng_tls.state = seed if seed else ops.THE_RNG_SEED


class FlannBasedMatcher:
    """cv2.FlannBasedMatcher(dict(algorithm=1, trees=5), dict(checks=50)) as
    built at v3:206-212: OpenCV's randomized kd-forest (FLANN_INDEX_KDTREE)
    built over the train descriptors and searched approximately with `checks`
    leaf visits, on the GPU (ops.flann_knn / dvo_flann_knn; oracle/flann.cpp
    restates it).  The trees come from cv::theRNG(), carried per thread across
    calls as in OpenCV.  DMatch.distance is sqrt(float32) of FLANN's squared
    L2 distance, as FlannBasedMatcher::convertToDMatches does for float
    descriptors, so the 0.75 ratio test (v3:227) compares distances.

    OpenCV 4.x only: the FLANN bundled with OpenCV 3.2 drew its trees from
    std::rand / std::random_shuffle, which are not restated, so with
    OPENCV_SEMANTICS == "3.2" the constructor raises cv.error rather than
    silently building 4.x trees.  Parity is against oracle/flann.cpp (the
    restatement); against OpenCV's FLANN itself it is unpinned (no cv2 here)."""

    def __init__(self, indexParams=None, searchParams=None):
        if opencv_semantics(OPENCV_SEMANTICS) == 1:
            raise error("FlannBasedMatcher reproduces OpenCV 4.x's FLANN (cv::theRNG trees); the OpenCV 3.2 "
                        "FLANN (std::rand trees) is not implemented -- unset DVO_OPENCV_SEMANTICS=3.2 for flann mode")
        self.indexParams = dict(indexParams or {})
        self.searchParams = dict(searchParams or {})
        if self.indexParams.get("algorithm", 1) != 1:
            raise error("only FLANN_INDEX_KDTREE (algorithm=1) is implemented (the reference's choice, v3:207)")
        self.trees = int(self.indexParams.get("trees", 4))        # KDTreeIndexParams default
        self.checks = int(self.searchParams.get("checks", 32))    # SearchParams default
        if float(self.searchParams.get("eps", 0.0)) != 0.0 or self.checks < 1:
            raise error("only eps=0 and checks >= 1 are implemented")

    def knnMatch(self, queryDescriptors, trainDescriptors, k, mask=None, compactResult=False):
        if mask is not None:
            raise error("match masks are not supported")
        q, t = _float_desc(queryDescriptors), _float_desc(trainDescriptors)
        if len(q) == 0 or len(t) == 0:  # DescriptorMatcher::knnMatch returns before training
            return []
        if q.shape[1] != t.shape[1]:
            raise error("(-215:Assertion failed) query and train descriptors differ in length")
        if int(k) > len(t):
            raise error("(-215:Assertion failed) (size_t)knn <= index_->size() in function 'runKnnSearch_'")
        try:
            idx, dist, st = ops.flann_knn(q, t, int(k), self.trees, self.checks, _the_rng())
        except DVOError as e:
            raise error(str(e)) from e
        _rng_tls.state = st
        dist = np.sqrt(dist.astype(np.float32))
        out = []
        for qi in range(len(q)):
            out.append([DMatch(qi, int(idx[qi, s]), 0, float(dist[qi, s])) for s in range(int(k)) if idx[qi, s] >= 0])
        return [r for r in out if r] if compactResult else out


def findEssentialMat(points1, points2, cameraMatrix=None, method=RANSAC, prob=0.999, threshold=1.0, maxIters=1000,
                     mask=None, **kw):
    """(E, mask) like cv2.findEssentialMat(..., RANSAC); (None, None) where OpenCV returns an empty E."""
    if cameraMatrix is None:
        raise error("cameraMatrix is required")
    if method != RANSAC:
        raise error("only method=cv.RANSAC is implemented (v3:299)")
    p1 = np.asarray(points1, np.float64).reshape(-1, 2)
    p2 = np.asarray(points2, np.float64).reshape(-1, 2)
    if len(p1) != len(p2):
        raise error("(-215:Assertion failed) npoints >= 0 && points2.checkVector(2) == npoints")
    try:
        return ops.find_essential_mat(p1, p2, cameraMatrix, prob, threshold, maxIters)
    except DVOError as e:
        if e.code in (-3, -6):  # fewer than 5 points / no model: OpenCV returns an empty E
            return None, None
        raise error(str(e)) from e


def recoverPose(E, points1, points2, cameraMatrix=None, R=None, t=None, mask=None, distanceThresh=50.0, **kw):
    """(retval, R, t, mask) like cv2.recoverPose(E, points1, points2, cameraMatrix)."""
    if E is None or np.asarray(E).size == 0:
        raise error("(-215:Assertion failed) E.cols == 3 && E.rows == 3 in function 'decomposeEssentialMat'")
    E = np.asarray(E, np.float64)
    if E.shape != (3, 3):
        raise error("(-215:Assertion failed) E.cols == 3 && E.rows == 3 in function 'decomposeEssentialMat'")
    if cameraMatrix is None:
        raise error("cameraMatrix is required")
    p1 = np.asarray(points1, np.float64).reshape(-1, 2)
    p2 = np.asarray(points2, np.float64).reshape(-1, 2)
    try:
        return ops.recover_pose(E, p1, p2, cameraMatrix, distanceThresh, mask)
    except DVOError as e:
        raise error(str(e)) from e


def triangulatePoints(projMatr1, projMatr2, projPoints1, projPoints2, points4D=None):
    if projMatr1 is None or projMatr2 is None:
        raise error("(-215:Assertion failed) projection matrices must be 3x4")
    P1 = np.asarray(projMatr1, np.float64)
    P2 = np.asarray(projMatr2, np.float64)
    if P1.shape != (3, 4) or P2.shape != (3, 4):
        raise error("(-215:Assertion failed) projection matrices must be 3x4")
    try:
        return ops.triangulate_points(P1, P2, projPoints1, projPoints2)
    except DVOError as e:
        raise error(str(e)) from e


# ---- host-side helpers outside the GPU hot path ------------------------------
def _gray(image):
    img = np.asarray(image)
    if img.ndim == 3 and img.shape[2] == 3:
        return cvtColor(img, COLOR_BGR2GRAY)
    if img.ndim != 2 or img.dtype != np.uint8:
        raise error("expected a mono8 or BGR8 image")
    return img


def cvtColor(src, code):
    """COLOR_BGR2GRAY with OpenCV's 8-bit fixed point (R 4899, G 9617, B 1868, >> 14)."""
    src = np.asarray(src)
    if code == COLOR_BGR2GRAY:
        if src.ndim == 2:
            return src.copy()
        b = src[..., 0].astype(np.int32)
        g = src[..., 1].astype(np.int32)
        r = src[..., 2].astype(np.int32)
        return ((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)
    if code == COLOR_GRAY2BGR:
        return np.repeat(src[..., None], 3, axis=2)
    raise error(f"cvtColor code {code} not supported")


def imdecode(buf, flags=IMREAD_COLOR):
    """JPEG/PNG decode (PIL) to BGR8 (IMREAD_COLOR) or mono8; None on failure, like cv2."""
    import io
    try:
        from PIL import Image
        im = Image.open(io.BytesIO(np.asarray(buf, np.uint8).tobytes()))
        if flags == IMREAD_GRAYSCALE:
            return np.asarray(im.convert("L"))
        return np.ascontiguousarray(np.asarray(im.convert("RGB"))[..., ::-1])
    except Exception:
        return None


def getOptimalNewCameraMatrix(cameraMatrix, distCoeffs, imageSize, alpha, newImgSize=None, centerPrincipalPoint=False):
    """(newK, validPixROI) like cv2 (v3:117).  The ROI, which the reference
    discards, is reported as the full new image."""
    if centerPrincipalPoint:
        raise error("centerPrincipalPoint=True is not implemented (the reference uses the default)")
    w, h = imageSize
    nw, nh = (w, h) if newImgSize is None or newImgSize[0] * newImgSize[1] == 0 else newImgSize
    try:
        K = ops.get_optimal_new_camera_matrix(cameraMatrix, distCoeffs, (w, h), alpha, (nw, nh))
    except DVOError as e:
        raise error(str(e)) from e
    return K, (0, 0, int(nw), int(nh))


class _UndistortCache:
    """cv.undistort builds its remap table per call; the table only depends on
    (K, dist, newK, size), so it is built once on the device and reused."""

    def __init__(self):
        self.key = None
        self.u = None

    def get(self, K, dist, newK, w, h):
        key = (np.asarray(K, np.float64).tobytes(), np.asarray(dist, np.float64).tobytes(),
               None if newK is None else np.asarray(newK, np.float64).tobytes(), w, h)
        if key != self.key:
            self.u = ops.Undistorter(K, dist, newK, w, h)
            self.key = key
        return self.u


_undistort_cache = _UndistortCache()


def undistort(src, cameraMatrix, distCoeffs, dst=None, newCameraMatrix=None):
    """remap(src, initUndistortRectifyMap(K, dist, I, newK), INTER_LINEAR,
    BORDER_CONSTANT) on the GPU (v3:120)."""
    img = np.asarray(src)
    if img.dtype != np.uint8 or img.ndim != 2:
        raise error("undistort is implemented for mono8 images (the reference undistorts the gray frame, v3:133-135)")
    h, w = img.shape
    d = np.asarray(distCoeffs if distCoeffs is not None else np.zeros(5), np.float64).ravel()
    try:
        out = _undistort_cache.get(cameraMatrix, d, newCameraMatrix, w, h).image(img)
    except DVOError as e:
        raise error(str(e)) from e
    if dst is not None:
        np.copyto(dst, out)
        return dst
    return out


_CIRCLE3 = [(dx, dy) for dx in range(-3, 4) for dy in range(-3, 4) if round((dx * dx + dy * dy) ** 0.5) == 3]


def drawKeypoints(image, keypoints, outImage=None, color=(0, 255, 0), flags=0):
    """BGR copy of `image` with a radius-3 circle at every keypoint (DEFAULT flag).
    The reference computes and discards this image (v3:375, D6)."""
    img = np.asarray(image)
    out = np.repeat(img[..., None], 3, axis=2).copy() if img.ndim == 2 else img.copy()
    arr = keypoints.array if isinstance(keypoints, KeyPoints) else None
    if arr is not None:
        xs = np.rint(arr["x"]).astype(np.int64)
        ys = np.rint(arr["y"]).astype(np.int64)
    else:
        xs = np.array([int(round(k.pt[0])) for k in keypoints], np.int64)
        ys = np.array([int(round(k.pt[1])) for k in keypoints], np.int64)
    h, w = out.shape[:2]
    col = np.asarray(color[:3], np.uint8)
    for dx, dy in _CIRCLE3:
        x, y = xs + dx, ys + dy
        ok = (x >= 0) & (x < w) & (y >= 0) & (y < h)
        out[y[ok], x[ok]] = col
    return out


class SIFT:
    """cv2.SIFT with SIFT_create()'s defaults (v3:100), on the GPU
    (dvo_sift_detect_and_compute): keypoints and float32[N, 128] descriptors
    for the float k-NN matchers of the sift / knn_sift / flann modes."""

    def __init__(self, nfeatures=0, nOctaveLayers=3, contrastThreshold=0.04, edgeThreshold=10, sigma=1.6):
        if (nfeatures != 0 or nOctaveLayers != 3 or not np.isclose(contrastThreshold, 0.04)
                or not np.isclose(edgeThreshold, 10) or not np.isclose(sigma, 1.6)):
            raise error("only the SIFT_create() defaults are implemented (the reference uses them, v3:100)")

    def detectAndCompute(self, image, mask, descriptors=None, useProvidedKeypoints=False):
        if mask is not None:
            raise error("SIFT masks are not supported (the reference passes None, v3:373)")
        if useProvidedKeypoints:
            raise error("useProvidedKeypoints is not supported")
        img = _gray(image)
        try:
            kps, desc = ops.sift_detect_and_compute(img)
        except DVOError as e:
            raise error(str(e)) from e
        return KeyPoints(kps), (desc if len(kps) else None)

    def detect(self, image, mask=None):
        return self.detectAndCompute(image, mask)[0]

    def descriptorSize(self):
        return 128


def SIFT_create(nfeatures=0, nOctaveLayers=3, contrastThreshold=0.04, edgeThreshold=10, sigma=1.6):
    return SIFT(nfeatures, nOctaveLayers, contrastThreshold, edgeThreshold, sigma)


class SURF:
    """cv2.xfeatures2d.SURF (v3:104, SURF_create(400)) on the GPU
    (dvo_surf_detect_and_compute): keypoints and float32[N, 64] descriptors for
    the surf mode's NORM_L1 knnMatch (v3:215)."""

    def __init__(self, hessianThreshold=100, nOctaves=4, nOctaveLayers=3, extended=False, upright=False):
        if nOctaves != 4 or nOctaveLayers != 3 or extended or upright:
            raise error("only nOctaves 4, nOctaveLayers 3, extended False, upright False are implemented "
                        "(the reference's SURF_create(400), v3:104)")
        if not hessianThreshold >= 0:
            raise error("hessianThreshold must be >= 0")
        self.hessianThreshold = float(hessianThreshold)

    def detectAndCompute(self, image, mask, descriptors=None, useProvidedKeypoints=False):
        if mask is not None:
            raise error("SURF masks are not supported (the reference passes None, v3:373)")
        if useProvidedKeypoints:
            raise error("useProvidedKeypoints is not supported")
        img = _gray(image)
        try:
            kps, desc = ops.surf_detect_and_compute(img, self.hessianThreshold)
        except DVOError as e:
            raise error(str(e)) from e
        return KeyPoints(kps), (desc if len(kps) else None)

    def detect(self, image, mask=None):
        return self.detectAndCompute(image, mask)[0]

    def descriptorSize(self):
        return 64

    def getHessianThreshold(self):
        return self.hessianThreshold


def SURF_create(hessianThreshold=100, nOctaves=4, nOctaveLayers=3, extended=False, upright=False):
    return SURF(hessianThreshold, nOctaves, nOctaveLayers, extended, upright)


class _XFeatures2d:
    """cv2.xfeatures2d: SIFT (v3:100) and SURF (v3:104) on the GPU."""

    @staticmethod
    def SIFT_create(*a, **k):
        return SIFT_create(*a, **k)

    @staticmethod
    def SURF_create(*a, **k):
        return SURF_create(*a, **k)


xfeatures2d = _XFeatures2d()


def imshow(*a, **k):  # visualisation helpers are out of scope
    raise error("imshow is not available (no GUI)")


def waitKey(*a, **k):
    return -1


def imwrite(path, img):
    from PIL import Image
    arr = np.asarray(img)
    if arr.ndim == 3:
        arr = arr[..., ::-1]
    Image.fromarray(arr).save(path)
    return True
