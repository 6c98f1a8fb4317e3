"""numpy-level wrappers of the per-call C-ABI entry points (include/dvo.h).

Each function replaces one OpenCV operator of the reference's hot path and
mirrors its argument meaning, output layout and failure points:

  detect_and_compute   cv::ORB::detectAndCompute          visual_odometry_v3.py:373
  bf_match             cv::BFMatcher(NORM_HAMMING).match  visual_odometry_v3.py:75, :219
  find_essential_mat   cv::findEssentialMat(RANSAC)       visual_odometry_v3.py:297-300
  recover_pose         cv::recoverPose                    visual_odometry_v3.py:303-306
  triangulate_points   cv::triangulatePoints              visual_odometry_v3.py:265
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._native import (DMATCH_DTYPE, DVO_ECAP, DVO_OK, KEYPOINT_DTYPE, Context, DVOError, orb_params, ptr)


def _ctx(ctx):
    return ctx if ctx is not None else Context.default()


def detect_and_compute(img: np.ndarray, nfeatures: int = 500, fast_threshold: int = 20, ctx=None):
    """ORB keypoints (structured KEYPOINT_DTYPE array) and uint8[N, 32] descriptors."""
    c = _ctx(ctx)
    img = np.ascontiguousarray(img)
    if img.dtype != np.uint8 or img.ndim != 2:
        raise DVOError(-1, "detect_and_compute expects a mono8 image (uint8[H, W])")
    h, w = img.shape
    prm = orb_params(nfeatures=nfeatures, fast_threshold=fast_threshold)
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
def test_retain_best(resp, n_points, depth=-1, ctx=None):
    c = _ctx(ctx)
    resp = np.ascontiguousarray(resp, np.float32)
    perm = np.zeros(max(len(resp), 1), np.int32)
    k = ctypes.c_int()
    c.check(c.lib.dvo_test_retain_best(c.h, ptr(resp), len(resp), int(n_points), int(depth), ptr(perm),
                                       ctypes.byref(k)))
    return perm[:k.value].copy()


def test_update_num_iters(p, eps, model_points, max_iters, ctx=None):
    c = _ctx(ctx)
    eps = np.ascontiguousarray(eps, np.float64)
    out = np.zeros(max(len(eps), 1), np.int32)
    c.check(c.lib.dvo_test_update_num_iters(c.h, float(p), ptr(eps), len(eps), int(model_points), int(max_iters),
                                            ptr(out)))
    return out[:len(eps)]


def test_five_point(q1, q2, ctx=None):
    c = _ctx(ctx)
    q1 = np.ascontiguousarray(q1, np.float64).reshape(10)
    q2 = np.ascontiguousarray(q2, np.float64).reshape(10)
    models = np.zeros(90, np.float64)
    n = ctypes.c_int()
    c.check(c.lib.dvo_test_five_point(c.h, ptr(q1), ptr(q2), ptr(models), ctypes.byref(n)))
    return models[:9 * n.value].reshape(n.value, 3, 3).copy()
