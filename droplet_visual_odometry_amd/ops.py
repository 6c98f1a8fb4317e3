"""numpy-level wrappers of the per-call C-ABI entry points (include/dvo.h).

Each function replaces one OpenCV operator of the reference's hot path and
mirrors its argument meaning, output layout and failure points:

  detect_and_compute   cv::ORB::detectAndCompute          visual_odometry_v3.py:373
  sift_detect_and_compute  cv::SIFT::detectAndCompute    visual_odometry_v3.py:100, :373
  bf_match             cv::BFMatcher(NORM_HAMMING).match  visual_odometry_v3.py:75, :219
  bf_knn_float         cv::BFMatcher(NORM_L1).knnMatch / .match, FLANN knnMatch
                                                          visual_odometry_v3.py:99-106, :200-215
  find_essential_mat   cv::findEssentialMat(RANSAC)       visual_odometry_v3.py:297-300
  recover_pose         cv::recoverPose                    visual_odometry_v3.py:303-306
  triangulate_points   cv::triangulatePoints              visual_odometry_v3.py:265
  get_optimal_new_camera_matrix, Undistorter
                       cv::getOptimalNewCameraMatrix, cv::undistort  v3:117, v3:120
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._native import (DMATCH_DTYPE, DVO_ECAP, DVO_OK, KEYPOINT_DTYPE, PAIR_RECORD_DTYPE, Context, DVOError, StreamConfig,
                      load_library, orb_params, ptr)


def _ctx(ctx):
    return ctx if ctx is not None else Context.default()


def detect_and_compute(img: np.ndarray, nfeatures: int = 500, fast_threshold: int = 20, opencv="4.x", ctx=None):
    """ORB keypoints (structured KEYPOINT_DTYPE array) and uint8[N, 32] descriptors.
    opencv: "4.x" (default) or "3.2" semantics (include/dvo.h DVO_OPENCV_*)."""
    c = _ctx(ctx)
    img = np.ascontiguousarray(img)
    if img.dtype != np.uint8 or img.ndim != 2:
        raise DVOError(-1, "detect_and_compute expects a mono8 image (uint8[H, W])")
    h, w = img.shape
    prm = orb_params(nfeatures=nfeatures, fast_threshold=fast_threshold, opencv=opencv)
    cap = nfeatures + 512
    while True:
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_int()
        rc = c.lib.dvo_orb_detect_and_compute(c.h, ctypes.byref(prm), ptr(img), w, h, img.strides[0], ptr(kps),
                                              ptr(desc), cap, ctypes.byref(n))
        if rc == DVO_ECAP and n.value > cap:
            cap = n.value
            continue
        c.check(rc)
        return kps[:n.value].copy(), desc[:n.value].copy()


def sift_detect_and_compute(img: np.ndarray, ctx=None):
    """SIFT_create().detectAndCompute(img, None): keypoints (KEYPOINT_DTYPE, in
    OpenCV's removeDuplicatedSorted order) and float32[N, 128] descriptors."""
    c = _ctx(ctx)
    img = np.ascontiguousarray(img)
    if img.dtype != np.uint8 or img.ndim != 2:
        raise DVOError(-1, "sift_detect_and_compute expects a mono8 image (uint8[H, W])")
    h, w = img.shape
    cap = 8192
    while True:
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 128), np.float32)
        n = ctypes.c_int()
        rc = c.lib.dvo_sift_detect_and_compute(c.h, ptr(img), w, h, img.strides[0], ptr(kps), ptr(desc), cap,
                                               ctypes.byref(n))
        if rc == DVO_ECAP and n.value > cap:
            cap = n.value
            continue
        c.check(rc)
        return kps[:n.value].copy(), desc[:n.value].copy()


def surf_detect_and_compute(img: np.ndarray, hessian_threshold: float = 400.0, ctx=None):
    """xfeatures2d.SURF_create(hessian_threshold).detectAndCompute(img, None) on
    the GPU (dvo_surf_detect_and_compute): KEYPOINT_DTYPE array (OpenCV's
    KeypointGreater order) and float32[N, 64] descriptors."""
    c = _ctx(ctx)
    img = np.ascontiguousarray(img)
    if img.dtype != np.uint8 or img.ndim != 2:
        raise DVOError(-1, "surf_detect_and_compute expects a mono8 image (uint8[H, W])")
    h, w = img.shape
    cap = 8192
    while True:
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 64), np.float32)
        n = ctypes.c_int()
        rc = c.lib.dvo_surf_detect_and_compute(c.h, ptr(img), w, h, img.strides[0], float(hessian_threshold), ptr(kps),
                                               ptr(desc), cap, ctypes.byref(n))
        if rc == DVO_ECAP and n.value > cap:
            cap = n.value
            continue
        c.check(rc)
        return kps[:n.value].copy(), desc[:n.value].copy()


def bf_match(dq: np.ndarray, dt: np.ndarray, cross_check: int = 1, ctx=None) -> np.ndarray:
    """DMATCH_DTYPE array in queryIdx order (OpenCV's output order)."""
    c = _ctx(ctx)
    dq = np.ascontiguousarray(dq, np.uint8).reshape(-1, 32)
    dt = np.ascontiguousarray(dt, np.uint8).reshape(-1, 32)
    out = np.zeros(max(len(dq), 1), DMATCH_DTYPE)
    m = ctypes.c_int()
    c.check(c.lib.dvo_bf_match_hamming(c.h, ptr(dq), len(dq), ptr(dt), len(dt), int(cross_check), ptr(out), len(out),
                                       ctypes.byref(m)))
    return out[:m.value].copy()


NORM_L1, NORM_L2SQR = 0, 1


def bf_knn_float(dq: np.ndarray, dt: np.ndarray, k: int = 2, norm: int = NORM_L1, ctx=None):
    """k nearest trains of each float query: (train_idx int32[nq, k], dist
    float32[nq, k]) in OpenCV's order (ascending distance, lower train index
    first on ties); -1 / FLT_MAX pad queries with fewer than k trains.
    norm NORM_L1 (BFMatcher(NORM_L1)) or NORM_L2SQR (FLANN's squared L2)."""
    c = _ctx(ctx)
    dq = np.ascontiguousarray(dq, np.float32)
    dt = np.ascontiguousarray(dt, np.float32)
    if dq.ndim != 2 or dt.ndim != 2 or (len(dt) and dt.shape[1] != dq.shape[1]):
        raise DVOError(-1, "descriptors must be float32[n, dim] with the same dim")
    nq, nt, dim = dq.shape[0], dt.shape[0], dq.shape[1]
    idx = np.zeros((max(nq, 1), k), np.int32)
    dist = np.zeros((max(nq, 1), k), np.float32)
    c.check(c.lib.dvo_bf_knn_float(c.h, ptr(dq), nq, ptr(dt), nt, dim, int(k), int(norm), ptr(idx), ptr(dist)))
    return idx[:nq].copy(), dist[:nq].copy()


THE_RNG_SEED = 0xFFFFFFFF  # cv::theRNG() of a fresh thread (cv::RNG() state)


def flann_knn(dq: np.ndarray, dt: np.ndarray, k: int = 2, trees: int = 5, checks: int = 50,
              rng_state: int = THE_RNG_SEED, ctx=None):
    """FlannBasedMatcher(KDTREE trees, checks).knnMatch(dq, dt, k) on the GPU
    (dvo_flann_knn): (train_idx int32[nq, k], squared L2 float32[nq, k], the
    cv::theRNG() state after the call).  The randomized kd-forest and its
    approximate search reproduce OpenCV's, given the theRNG state before."""
    c = _ctx(ctx)
    dq = np.ascontiguousarray(dq, np.float32)
    dt = np.ascontiguousarray(dt, np.float32)
    if dq.ndim != 2 or dt.ndim != 2 or (len(dt) and len(dq) and dt.shape[1] != dq.shape[1]):
        raise DVOError(-1, "descriptors must be float32[n, dim] with the same dim")
    nq, nt, dim = dq.shape[0], dt.shape[0], dq.shape[1] if dq.size else dt.shape[1]
    idx = np.zeros((max(nq, 1), k), np.int32)
    dist = np.zeros((max(nq, 1), k), np.float32)
    st = ctypes.c_uint64(int(rng_state))
    c.check(c.lib.dvo_flann_knn(c.h, ptr(dq), nq, ptr(dt), nt, dim, int(k), int(trees), int(checks), ctypes.byref(st),
                                ptr(idx), ptr(dist)))
    return idx[:nq].copy(), dist[:nq].copy(), int(st.value)


def _pts(p):
    p = np.ascontiguousarray(np.asarray(p, dtype=np.float64).reshape(-1, 2))
    return p


def find_essential_mat(p1, p2, K, prob=0.999, threshold=1.0, max_iters=1000, ctx=None):
    """(E float64[3k, 3], mask uint8[M, 1]).  Raises DVOError where OpenCV returns an empty E."""
    c = _ctx(ctx)
    p1, p2 = _pts(p1), _pts(p2)
    if len(p1) != len(p2):
        raise DVOError(-1, "findEssentialMat: point arrays differ in length")
    K = np.ascontiguousarray(K, np.float64).reshape(9)
    m = len(p1)
    E = np.zeros(90, np.float64)
    rows = ctypes.c_int()
    mask = np.zeros(max(m, 1), np.uint8)
    c.check(c.lib.dvo_find_essential_mat(c.h, ptr(p1), ptr(p2), m, ptr(K), float(prob), float(threshold),
                                         int(max_iters), ptr(E), ctypes.byref(rows), ptr(mask)))
    return E[:3 * rows.value].reshape(rows.value, 3).copy(), mask[:m].reshape(m, 1).copy()


def recover_pose(E, p1, p2, K, distance_thresh=50.0, mask=None, ctx=None):
    """(good, R float64[3,3], t float64[3,1], mask uint8[M,1] of 0/255)."""
    c = _ctx(ctx)
    E = np.ascontiguousarray(E, np.float64)
    if E.ndim != 2 or E.shape[1] != 3 or E.shape[0] != 3:
        raise DVOError(-1, "recoverPose: E must be 3x3")
    p1, p2 = _pts(p1), _pts(p2)
    m = len(p1)
    K = np.ascontiguousarray(K, np.float64).reshape(9)
    R = np.zeros(9, np.float64)
    t = np.zeros(3, np.float64)
    mo = np.zeros(max(m, 1), np.uint8)
    good = ctypes.c_int()
    mk = None if mask is None else np.ascontiguousarray(np.asarray(mask).reshape(-1), np.uint8)
    c.check(c.lib.dvo_recover_pose(c.h, ptr(E), 3, ptr(p1), ptr(p2), m, ptr(K), float(distance_thresh), ptr(mk),
                                   ptr(R), ptr(t), ptr(mo), ctypes.byref(good)))
    return good.value, R.reshape(3, 3), t.reshape(3, 1), mo[:m].reshape(m, 1).copy()


def triangulate_points(P1, P2, x1, x2, ctx=None) -> np.ndarray:
    """float64[4, K] homogeneous points; x1/x2 are 2 x K (or K x 2 with channels)."""
    c = _ctx(ctx)
    x1 = np.asarray(x1, np.float64)
    x2 = np.asarray(x2, np.float64)
    if x1.ndim == 2 and x1.shape[0] != 2 and x1.shape[1] == 2:
        x1, x2 = x1.T, x2.T
    x1 = np.ascontiguousarray(x1.reshape(2, -1))
    x2 = np.ascontiguousarray(x2.reshape(2, -1))
    k = x1.shape[1]
    X = np.zeros((4, k), np.float64)
    c.check(c.lib.dvo_triangulate_points(c.h, ptr(np.ascontiguousarray(P1, np.float64)),
                                         ptr(np.ascontiguousarray(P2, np.float64)), ptr(x1), ptr(x2), k, ptr(X)))
    return X


# ---- device test hooks --------------------------------------------------------
def test_retain_best(resp, n_points, depth=-1, opencv="4.x", ctx=None):
    from ._native import opencv_semantics
    c = _ctx(ctx)
    resp = np.ascontiguousarray(resp, np.float32)
    perm = np.zeros(max(len(resp), 1), np.int32)
    k = ctypes.c_int()
    c.check(c.lib.dvo_test_retain_best(c.h, ptr(resp), len(resp), int(n_points), int(depth),
                                       opencv_semantics(opencv), ptr(perm), ctypes.byref(k)))
    return perm[:k.value].copy()


def test_update_num_iters(p, eps, model_points, max_iters, ctx=None):
    c = _ctx(ctx)
    eps = np.ascontiguousarray(eps, np.float64)
    out = np.zeros(max(len(eps), 1), np.int32)
    c.check(c.lib.dvo_test_update_num_iters(c.h, float(p), ptr(eps), len(eps), int(model_points), int(max_iters),
                                            ptr(out)))
    return out[:len(eps)]


def test_ransac_subsets(m, n, ctx=None):
    """Device getSubset draws for n hypotheses over m correspondences (n x 5)."""
    c = _ctx(ctx)
    idx = np.zeros((n, 5), np.int32)
    c.check(c.lib.dvo_test_ransac_subsets(c.h, int(m), int(n), ptr(idx)))
    return idx


def test_ransac_replay(nmod, cnt, m, prob=0.999, max_iters=1000, ctx=None):
    """Device RANSAC bookkeeping: (iterations, niters, max good, best h, best model)."""
    c = _ctx(ctx)
    nmod = np.ascontiguousarray(nmod, np.int32)
    cnt = np.ascontiguousarray(cnt, np.int32).reshape(-1, 10)
    out = np.zeros(5, np.int32)
    c.check(c.lib.dvo_test_ransac_replay(c.h, ptr(nmod), ptr(cnt), len(nmod), int(m), float(prob), int(max_iters),
                                         ptr(out)))
    return tuple(int(v) for v in out)


def test_five_point(q1, q2, ctx=None):
    c = _ctx(ctx)
    q1 = np.ascontiguousarray(q1, np.float64).reshape(10)
    q2 = np.ascontiguousarray(q2, np.float64).reshape(10)
    models = np.zeros(90, np.float64)
    n = ctypes.c_int()
    c.check(c.lib.dvo_test_five_point(c.h, ptr(q1), ptr(q2), ptr(models), ctypes.byref(n)))
    return models[:9 * n.value].reshape(n.value, 3, 3).copy()


def test_sampson(E, pts, t, ctx=None):
    """Device f32 Sampson decision (1 / 0 / -1 undecided) and the f64 test, per point."""
    c = _ctx(ctx)
    E = np.ascontiguousarray(E, np.float64).reshape(9)
    pts = np.ascontiguousarray(pts, np.float64).reshape(-1, 4)
    n = len(pts)
    dec = np.zeros(n, np.int8)
    ex = np.zeros(n, np.uint8)
    c.check(c.lib.dvo_test_sampson(c.h, ptr(E), ptr(pts), n, float(t), ptr(dec), ptr(ex)))
    return dec, ex.astype(bool)


# ---- image pre-processing (visual_odometry_v3.py:110-135) ----
def get_optimal_new_camera_matrix(K, dist, size, alpha=1.0, new_size=None) -> np.ndarray:
    """cv.getOptimalNewCameraMatrix(K, dist, size, alpha, new_size)[0] (v3:117)."""
    lib = load_library()
    d = np.ascontiguousarray(np.asarray(dist, np.float64).ravel())
    w, h = size
    nw, nh = (w, h) if new_size is None else new_size
    out = np.zeros(9, np.float64)
    rc = lib.dvo_get_optimal_new_camera_matrix(ptr(np.ascontiguousarray(K, np.float64).reshape(9)), ptr(d), len(d),
                                               int(w), int(h), float(alpha), int(nw), int(nh), ptr(out))
    if rc != DVO_OK:
        raise DVOError(rc, "getOptimalNewCameraMatrix: bad arguments (distortion needs 0, 4, 5, 8 or 12 values)")
    return out.reshape(3, 3)


class Undistorter:
    """cv.undistort(img, K, dist, None, newK) (v3:120) with the remap table built
    once on the device.  image(): host in/out; apply(): device frames."""

    def __init__(self, K, dist, newK, width: int, height: int, ctx=None):
        self.ctx = _ctx(ctx)
        self.w, self.h = int(width), int(height)
        d = np.ascontiguousarray(np.asarray(dist, np.float64).ravel())
        nk = None if newK is None else np.ascontiguousarray(newK, np.float64).reshape(9)
        h = ctypes.c_void_p()
        self.ctx.check(self.ctx.lib.dvo_undistort_create(self.ctx.h, ptr(np.ascontiguousarray(K, np.float64).reshape(9)),
                                                         ptr(d), len(d), ptr(nk), self.w, self.h, ctypes.byref(h)))
        self.h_ = h

    def image(self, img: np.ndarray) -> np.ndarray:
        img = np.ascontiguousarray(img, np.uint8)
        if img.shape != (self.h, self.w):
            raise DVOError(-1, f"image {img.shape} != undistorter size {(self.h, self.w)}")
        out = np.empty_like(img)
        self.ctx.check(self.ctx.lib.dvo_undistort_image(self.h_, ptr(img), img.strides[0], ptr(out), out.strides[0]))
        return out

    def apply(self, src, dst, hip_stream=None):
        """Remap n device frames (uint8 torch tensors [n, H, W], rows contiguous)
        on `hip_stream` (a non-NULL hipStream_t handle), by default ordered
        with torch's current stream."""
        n = src.shape[0]

        def call(st):
            self.ctx.check(self.ctx.lib.dvo_undistort_apply(self.h_, src.data_ptr(), n, src.stride(0), src.stride(1),
                                                            dst.data_ptr(), dst.stride(0), dst.stride(1),
                                                            ctypes.c_void_p(st)))
        if hip_stream:
            call(hip_stream)
        else:
            from .stream import ordered_side_stream
            with ordered_side_stream(src.device) as st:
                call(st)

    def map(self):
        xy = np.zeros((self.h, self.w, 2), np.int16)
        fr = np.zeros((self.h, self.w), np.uint16)
        self.ctx.check(self.ctx.lib.dvo_undistort_get_map(self.h_, ptr(xy), ptr(fr)))
        return xy, fr

    def close(self):
        if getattr(self, "h_", None):
            self.ctx.lib.dvo_undistort_destroy(self.h_)
            self.h_ = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PairStream:
    """One pair of host frames per call through the whole per-pair path
    (dvo_stream_pair): detectAndCompute of both frames, BFMatcher.match with
    crossCheck, findEssentialMat(RANSAC, prob, threshold, maxIters) and
    recoverPose (visual_odometry_v3.py:384-408 up to v3:303) in one
    synchronous library call, the 256-B pair record back.  With
    reuse_prev=True the previous frame is the last call's current frame and
    only the current one is detected.  The drop-in's fused path (D7) uses it;
    no torch involved."""

    def __init__(self, width, height, K, nfeatures=500, fast_threshold=20, cross_check=1, opencv="4.x", prob=0.999,
                 threshold=1.0, max_iters=1000, dist_thresh=50.0, ctx=None):
        self.ctx = _ctx(ctx)
        cfg = StreamConfig()
        cfg.width, cfg.height, cfg.max_frames = int(width), int(height), 2
        cfg.orb = orb_params(nfeatures=nfeatures, fast_threshold=fast_threshold, opencv=opencv)
        K = np.asarray(K, np.float64).reshape(9)
        for i in range(9):
            cfg.K[i] = float(K[i])
        cfg.prob, cfg.threshold, cfg.max_iters = float(prob), float(threshold), int(max_iters)
        cfg.cross_check, cfg.dist_thresh = int(cross_check), float(dist_thresh)
        h = ctypes.c_void_p()
        self.ctx.check(self.ctx.lib.dvo_stream_create(self.ctx.h, ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h
        self.width, self.height = int(width), int(height)

    def pair(self, prev_img, cur_img, reuse_prev=False) -> np.ndarray:
        cur = np.ascontiguousarray(cur_img, np.uint8)
        if cur.shape != (self.height, self.width):
            raise ValueError(f"frame shape {cur.shape} != {(self.height, self.width)}")
        prev = None
        if not reuse_prev:
            prev = np.ascontiguousarray(prev_img, np.uint8)
            if prev.shape != cur.shape:
                raise ValueError("previous and current frames differ in shape")
        rec = np.zeros(1, PAIR_RECORD_DTYPE)
        self.ctx.check(self.ctx.lib.dvo_stream_pair(self.h, ptr(prev), ptr(cur), self.width, int(bool(reuse_prev)),
                                                    ptr(rec)))
        return rec[0]

    def close(self):
        if getattr(self, "h", None):
            self.ctx.lib.dvo_stream_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
