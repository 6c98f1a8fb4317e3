"""TEST INFRASTRUCTURE ONLY — ctypes front end of the CPU oracle.

Wraps ``oracle/build/libdvo_oracle.so`` (built by ``oracle/Makefile``), the C++
restatement of the OpenCV operators on the reference's hot path
(scripts/visual_odometry_v3.py:297-306, :373, :219, :265; see oracle.h).
Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg import
this module; the product package never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libdvo_oracle.so")
_lib = None

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_kpp = np.ctypeslib.ndpointer(KEYPOINT_DTYPE, flags="C_CONTIGUOUS")
_ip = ctypes.POINTER(ctypes.c_int)
_c = ctypes.c_int
_d = ctypes.c_double


def build(force: bool = False) -> str:
    """make the oracle library (incremental: rebuilt when a source changed)."""
    subprocess.check_call(["make", "-s", "-C", _HERE] + (["-B"] if force else []))
    return _LIB_PATH


# OpenCV semantics of the ORB restatement (oracle.h ora_orb_detect_and_compute_v)
OCV4, OCV32 = 0, 1


def host_cpu():
    """(model name, tag): the host CPU's model and a hash of its model + flags."""
    import hashlib
    model, flags = "unknown", ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name") and model == "unknown":
                model = line.split(":", 1)[1].strip()
            elif line.startswith("flags") and not flags:
                flags = line.split(":", 1)[1].strip()
    except OSError:
        pass
    return model, hashlib.sha1((model + "|" + flags).encode()).hexdigest()[:10]


def use_native_build() -> str:
    """Switch this module to the -O3 -march=native build of the same sources
    (the CPU baseline; built here for this host CPU on first use).  Results
    are identical to the default build (no contraction, no fast-math)."""
    global _lib, _LIB_PATH
    tag = host_cpu()[1]
    path = os.path.join(_HERE, "build", f"libdvo_oracle_native_{tag}.so")
    if not os.path.exists(path):
        subprocess.check_call(["make", "-s", "-C", _HERE, "native", f"NATIVE_TAG={tag}"])
    if _LIB_PATH != path:
        _LIB_PATH, _lib = path, None
    return path


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        sig = {
            "ora_orb_level_sizes": [_c, _c, _c, _i32p],
            "ora_orb_features_per_level": [_c, _c, _i32p],
            "ora_orb_level_scales": [_c, _f32p],
            "ora_orb_pyramid": [_u8p, _c, _c, _c, _c, _c, _u8p],
            "ora_fast": [_u8p, _c, _c, _c, _c, _i32p, _c, _ip],
            "ora_retain_best": [_f32p, _c, _c, _i32p],
            "ora_retain_best_depth": [_f32p, _c, _c, _c, _i32p],
            "ora_orb_detect_and_compute": [_u8p, _c, _c, _c, _c, _kpp, _u8p, _c, _ip],
            "ora_orb_detect_and_compute_v": [_u8p, _c, _c, _c, _c, _c, _kpp, _u8p, _c, _ip],
            "ora_orb_pyramid_v": [_u8p, _c, _c, _c, _c, _c, _c, _u8p],
            "ora_retain_best_v": [_f32p, _c, _c, _c, _i32p],
            "ora_retain_best_depth_v": [_f32p, _c, _c, _c, _c, _i32p],
            "ora_bf_match_hamming": [_u8p, _c, _u8p, _c, _c, _i32p, _i32p, _f32p, _ip],
            "ora_bf_knn_float": [_f32p, _c, _f32p, _c, _c, _c, _c, _i32p, _f32p],
            "ora_flann_knn": [_f32p, _c, _f32p, _c, _c, _c, _c, _c, ctypes.POINTER(ctypes.c_uint64), _i32p, _f32p],
            "ora_find_essential": [_f64p, _f64p, _c, _f64p, _d, _d, _c, _f64p, _ip, _u8p, _ip],
            "ora_recover_pose": [_f64p, _f64p, _f64p, _c, _f64p, _d, ctypes.c_void_p, _f64p, _f64p, _u8p, _ip],
            "ora_triangulate": [_f64p, _f64p, _f64p, _f64p, _c, _f64p],
            "ora_five_point": [_f64p, _f64p, _f64p, _ip],
            "ora_jacobi_svd": [_f64p, _c, _c, _c, _f64p, _f64p],
            "ora_solve_poly": [_f64p, _c, _c, _f64p],
            "ora_ransac_update_num_iters": [_d, _d, _c, _c],
            "ora_ransac_subsets": [_c, _c, _i32p],
            "ora_ransac_replay": [_i32p, _i32p, _c, _c, _d, _c, _i32p],
            "ora_sift_detect_and_compute": [_u8p, _c, _c, _c, _kpp, _f32p, _c, _ip],
            "ora_surf_detect_and_compute": [_u8p, _c, _c, _c, ctypes.c_double, _kpp, _f32p, _c, _ip],
            "ora_get_optimal_new_camera_matrix": [_f64p, _f64p, _c, _c, _c, _d, _c, _c, _f64p],
            "ora_undistort": [_u8p, _c, _c, _c, _f64p, _f64p, _c, ctypes.c_void_p, _u8p, _c,
                              np.ctypeslib.ndpointer(np.int16, flags="C"), np.ctypeslib.ndpointer(np.uint16, flags="C")],
        }
        for name, args in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int
        L.ora_flann_rng_after.argtypes = [ctypes.c_uint64, _i32p, _c, _c]
        L.ora_flann_rng_after.restype = ctypes.c_uint64
        _lib = L
    return _lib


def level_sizes(w, h, nlevels=8):
    out = np.zeros(2 * nlevels, np.int32)
    lib().ora_orb_level_sizes(w, h, nlevels, out)
    return [(int(out[2 * l]), int(out[2 * l + 1])) for l in range(nlevels)]


def level_scales(nlevels=8):
    """The oracle's getScale per level (float32): keypoint coordinates of level l
    are float32(n) * level_scales()[l] (orb.cpp computeKeyPoints)."""
    out = np.zeros(nlevels, np.float32)
    lib().ora_orb_level_scales(nlevels, out)
    return out


def features_per_level(nfeatures, nlevels=8):
    out = np.zeros(nlevels, np.int32)
    lib().ora_orb_features_per_level(nfeatures, nlevels, out)
    return out.tolist()


def pyramid(img, nlevels=8, blurred=False, semantics=OCV4):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    sizes = level_sizes(w, h, nlevels)
    out = np.zeros(sum(a * b for a, b in sizes), np.uint8)
    lib().ora_orb_pyramid_v(img, w, h, w, nlevels, int(blurred), int(semantics), out)
    levels, off = [], 0
    for lw, lh in sizes:
        levels.append(out[off:off + lw * lh].reshape(lh, lw))
        off += lw * lh
    return levels


def fast(img, threshold=20):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = (w // 2 + 1) * (h // 2 + 1)
    buf = np.zeros(3 * cap, np.int32)
    n = ctypes.c_int()
    rc = lib().ora_fast(img, w, h, w, threshold, buf, cap, ctypes.byref(n))
    assert rc == 0
    return buf[:3 * n.value].reshape(-1, 3)


def retain_best(resp, n_points, depth=None, semantics=OCV4):
    resp = np.ascontiguousarray(resp, np.float32)
    perm = np.zeros(max(len(resp), 1), np.int32)
    if depth is None:
        k = lib().ora_retain_best_v(resp, len(resp), n_points, int(semantics), perm)
    else:
        k = lib().ora_retain_best_depth_v(resp, len(resp), n_points, depth, int(semantics), perm)
    return perm[:k]


def detect_and_compute(img, nfeatures=500, semantics=OCV4):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = 4 * nfeatures + 1024
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = ctypes.c_int()
    rc = lib().ora_orb_detect_and_compute_v(img, w, h, w, nfeatures, int(semantics), kps, desc, cap,
                                            ctypes.byref(n))
    assert rc == 0, rc
    return kps[:n.value].copy(), desc[:n.value].copy()


def sift_detect_and_compute(img):
    """SIFT_create().detectAndCompute(img, None): (KEYPOINT_DTYPE array, float32[n, 128])."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = 4096
    while True:
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 128), np.float32)
        n = ctypes.c_int()
        rc = lib().ora_sift_detect_and_compute(img, w, h, w, kps, desc, cap, ctypes.byref(n))
        if rc == -5:
            cap = n.value
            continue
        return kps[:n.value].copy(), desc[:n.value].copy()


def surf_detect_and_compute(img, hessian_threshold=400.0):
    """xfeatures2d.SURF_create(hessian_threshold).detectAndCompute(img, None):
    (KEYPOINT_DTYPE array, float32[n, 64])."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = 4096
    while True:
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 64), np.float32)
        n = ctypes.c_int()
        rc = lib().ora_surf_detect_and_compute(img, w, h, w, float(hessian_threshold), kps, desc, cap, ctypes.byref(n))
        if rc == -5:
            cap = n.value
            continue
        assert rc == 0, rc
        return kps[:n.value].copy(), desc[:n.value].copy()


def bf_match(dq, dt, mode=1):
    dq = np.ascontiguousarray(dq, np.uint8)
    dt = np.ascontiguousarray(dt, np.uint8)
    nq, nt = len(dq), len(dt)
    q = np.zeros(max(nq, 1), np.int32)
    t = np.zeros(max(nq, 1), np.int32)
    d = np.zeros(max(nq, 1), np.float32)
    m = ctypes.c_int()
    lib().ora_bf_match_hamming(dq.reshape(-1) if nq else np.zeros(32, np.uint8), nq,
                               dt.reshape(-1) if nt else np.zeros(32, np.uint8), nt, mode, q, t, d,
                               ctypes.byref(m))
    k = m.value
    return q[:k].copy(), t[:k].copy(), d[:k].copy()


def bf_knn_float(dq, dt, k=2, norm=0):
    """(train_idx int32[nq, k], dist float32[nq, k]); norm 0 = L1, 1 = squared L2."""
    dq = np.ascontiguousarray(dq, np.float32)
    dt = np.ascontiguousarray(dt, np.float32)
    nq, nt = len(dq), len(dt)
    dim = dq.shape[1] if dq.ndim == 2 else dt.shape[1]
    idx = np.zeros((max(nq, 1), k), np.int32)
    dist = np.zeros((max(nq, 1), k), np.float32)
    rc = lib().ora_bf_knn_float(dq.reshape(-1) if nq else np.zeros(dim, np.float32), nq,
                                dt.reshape(-1) if nt else np.zeros(dim, np.float32), nt, dim, k, norm, idx, dist)
    assert rc == 0, rc
    return idx[:nq].copy(), dist[:nq].copy()


def find_essential(p1, p2, K, prob=0.999, threshold=1.0, max_iters=1000):
    p1 = np.ascontiguousarray(p1, np.float64).reshape(-1)
    p2 = np.ascontiguousarray(p2, np.float64).reshape(-1)
    m = len(p1) // 2
    E = np.zeros(90, np.float64)
    rows = ctypes.c_int()
    mask = np.zeros(max(m, 1), np.uint8)
    iters = ctypes.c_int()
    rc = lib().ora_find_essential(p1, p2, m, np.ascontiguousarray(K, np.float64).reshape(-1), prob, threshold,
                                  max_iters, E, ctypes.byref(rows), mask, ctypes.byref(iters))
    if rc != 0:
        return None, None, iters.value
    return E[:rows.value * 3].reshape(rows.value, 3).copy(), mask[:m].copy(), iters.value


def recover_pose(E, p1, p2, K, dist_thresh=50.0, mask=None):
    p1 = np.ascontiguousarray(p1, np.float64).reshape(-1)
    p2 = np.ascontiguousarray(p2, np.float64).reshape(-1)
    m = len(p1) // 2
    R = np.zeros(9, np.float64)
    t = np.zeros(3, np.float64)
    mo = np.zeros(max(m, 1), np.uint8)
    good = ctypes.c_int()
    mk = None
    if mask is not None:
        mask = np.ascontiguousarray(mask, np.uint8).reshape(-1)
        mk = mask.ctypes.data_as(ctypes.c_void_p)
    lib().ora_recover_pose(np.ascontiguousarray(E, np.float64).reshape(-1), p1, p2, m,
                           np.ascontiguousarray(K, np.float64).reshape(-1), dist_thresh, mk, R, t, mo,
                           ctypes.byref(good))
    return good.value, R.reshape(3, 3), t.reshape(3, 1), mo[:m].copy()


def triangulate(P1, P2, x1, x2):
    x1 = np.ascontiguousarray(x1, np.float64)
    x2 = np.ascontiguousarray(x2, np.float64)
    k = x1.shape[1]
    X = np.zeros(4 * k, np.float64)
    lib().ora_triangulate(np.ascontiguousarray(P1, np.float64).reshape(-1),
                          np.ascontiguousarray(P2, np.float64).reshape(-1), x1.reshape(-1), x2.reshape(-1), k, X)
    return X.reshape(4, k)


def five_point(q1, q2):
    models = np.zeros(90, np.float64)
    n = ctypes.c_int()
    lib().ora_five_point(np.ascontiguousarray(q1, np.float64).reshape(-1),
                         np.ascontiguousarray(q2, np.float64).reshape(-1), models, ctypes.byref(n))
    return models[:9 * n.value].reshape(n.value, 3, 3).copy()


def jacobi_svd(A, full_u=False):
    """SVD of A (rows x cols) the way cv::SVD::compute does it (m >= n case only)."""
    A = np.asarray(A, np.float64)
    rows, cols = A.shape
    assert rows >= cols
    At = np.ascontiguousarray(A.T).reshape(-1).copy()
    W = np.zeros(cols)
    Vt = np.zeros(cols * cols)
    lib().ora_jacobi_svd(At, rows, cols, cols if full_u else 0, W, Vt)
    return W, At.reshape(cols, rows).T, Vt.reshape(cols, cols)


def solve_poly(coeffs, max_iters=300):
    coeffs = np.ascontiguousarray(coeffs, np.float64)
    n = len(coeffs) - 1
    roots = np.zeros(2 * n)
    k = lib().ora_solve_poly(coeffs, n, max_iters, roots)
    return roots[:2 * k].reshape(k, 2)


def ransac_update_num_iters(p, ep, model_points, max_iters):
    return lib().ora_ransac_update_num_iters(p, ep, model_points, max_iters)


def ransac_subsets(m, n):
    idx = np.zeros((max(n, 1), 5), np.int32)
    lib().ora_ransac_subsets(m, n, idx)
    return idx[:n]


def ransac_replay(nmod, cnt, m, prob=0.999, max_iters=1000):
    nmod = np.ascontiguousarray(nmod, np.int32)
    cnt = np.ascontiguousarray(cnt, np.int32).reshape(-1, 10)
    out = np.zeros(5, np.int32)
    lib().ora_ransac_replay(nmod, cnt, len(nmod), m, prob, max_iters, out)
    return tuple(int(v) for v in out)


def keypoints_to_points(kps):
    return np.stack([kps["x"], kps["y"]], axis=1).astype(np.float32)


def pair_pose(img_prev, img_cur, K, nfeatures=500, max_iters=1000, kp_prev=None, semantics=OCV4):
    """The full per-pair hot path (v3:384-408 minus the host pose tail) on the CPU.
    semantics OCV32: OpenCV 3.2's ORB pyramid / retainBest and BFMatcher
    cross check (mode 2)."""
    if kp_prev is None:
        kp_prev = detect_and_compute(img_prev, nfeatures, semantics)
    kp1, d1 = kp_prev
    kp2, d2 = detect_and_compute(img_cur, nfeatures, semantics)
    q, t, d = bf_match(d1, d2, 2 if semantics == OCV32 else 1)
    order = np.argsort(d, kind="stable")  # sorted(matches, key=distance), v3:221
    q, t = q[order], t[order]
    p1 = keypoints_to_points(kp1[q]).astype(np.float64)
    p2 = keypoints_to_points(kp2[t]).astype(np.float64)
    E, mask, iters = find_essential(p1, p2, K, max_iters=max_iters)
    out = dict(kp_prev=kp1, kp_cur=kp2, desc_cur=d2, q=q, t=t, p1=p1, p2=p2, E=E, mask=mask, iters=iters)
    if E is None or E.shape[0] != 3:
        out.update(R=None, t_unit=None, good=0)
        return out
    good, R, tv, _ = recover_pose(E, p1, p2, K)
    out.update(R=R, t_unit=tv, good=good)
    return out


def _euler_from_matrix_rxyz(R):
    """Gohlke euler_from_matrix(R, 'rxyz') (the `transformations` package call at
    visual_odometry_v3.py:334): i=2, j=1, k=0, parity, rotating frame."""
    import math
    i, j, k = 2, 1, 0
    cy = math.sqrt(R[i, i] * R[i, i] + R[j, i] * R[j, i])
    if cy > np.finfo(float).eps * 4.0:
        ax, ay, az = math.atan2(R[k, j], R[k, k]), math.atan2(-R[k, i], cy), math.atan2(R[j, i], R[i, i])
    else:
        ax, ay, az = math.atan2(-R[j, k], R[j, j]), math.atan2(-R[k, i], cy), 0.0
    ax, ay, az = -ax, -ay, -az
    return az, ay, ax


def _euler_matrix_sxyz(ai, aj, ak):
    """Gohlke euler_matrix(ai, aj, ak, 'sxyz') (visual_odometry_v3.py:140)."""
    import math
    si, sj, sk = math.sin(ai), math.sin(aj), math.sin(ak)
    ci, cj, ck = math.cos(ai), math.cos(aj), math.cos(ak)
    cc, cs, sc, ss = ci * ck, ci * sk, si * ck, si * sk
    M = np.identity(4)
    M[0, :3] = (cj * ck, sj * sc - cs, sj * cc + ss)
    M[1, :3] = (cj * sk, sj * ss + cc, sj * cs - sc)
    M[2, :3] = (-sj, cj * si, cj * ci)
    return M


def pose_tail(K, R, t, corners_prev, corners_cur, marker_length, P_prev, T_prev):
    """One pair of get_transformation_between_two_frames' tail (visual_odometry_v3.py:
    309-345) and the chain of previous_current_matching (v3:367):
    P_cur = K[R|t]; X = triangulatePoints(P_prev, P_cur, c_prev.T, c_cur.T);
    d = |X[:3,0]-X[:3,1]| (homogeneous, v3:283-289); s = L/d;
    T_rel = translation_matrix(t s) . euler_matrix(euler_from_matrix(R,'rxyz'),'sxyz').
    Returns (P_cur, T_rel, T_abs = T_prev . T_rel)."""
    K = np.asarray(K, np.float64)
    P_cur = K.dot(np.hstack((R, np.asarray(t, np.float64).reshape(3, 1))))
    X = triangulate(P_prev, P_cur, np.ascontiguousarray(np.asarray(corners_prev, np.float64).T),
                    np.ascontiguousarray(np.asarray(corners_cur, np.float64).T))
    d = float(np.sqrt((X[0, 0] - X[0, 1]) ** 2 + (X[1, 0] - X[1, 1]) ** 2 + (X[2, 0] - X[2, 1]) ** 2))
    s = marker_length / d
    T_rel = _euler_matrix_sxyz(*_euler_from_matrix_rxyz(np.asarray(R, np.float64)))
    T_rel[:3, 3] = np.asarray(t, np.float64).ravel() * s
    return P_cur, T_rel, np.asarray(T_prev, np.float64).dot(T_rel)


def get_optimal_new_camera_matrix(K, dist, w, h, alpha=1.0, new_size=None):
    """cv.getOptimalNewCameraMatrix(K, dist, (w, h), alpha, new_size) -> newK
    (visual_odometry_v3.py:117; restated in undistort.cpp)."""
    d = np.ascontiguousarray(np.asarray(dist, np.float64).ravel())
    nw, nh = (w, h) if new_size is None else new_size
    out = np.zeros(9, np.float64)
    lib().ora_get_optimal_new_camera_matrix(np.ascontiguousarray(K, np.float64).reshape(-1), d, len(d), w, h,
                                            float(alpha), nw, nh, out)
    return out.reshape(3, 3)


def undistort(img, K, dist, newK=None):
    """cv.undistort(img, K, dist, None, newK) (visual_odometry_v3.py:120) -> (dst, map_xy, map_frac)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    d = np.ascontiguousarray(np.asarray(dist, np.float64).ravel())
    dst = np.zeros_like(img)
    xy = np.zeros((h, w, 2), np.int16)
    fr = np.zeros((h, w), np.uint16)
    nk = None if newK is None else np.ascontiguousarray(newK, np.float64).reshape(-1)
    rc = lib().ora_undistort(img, w, h, img.strides[0], np.ascontiguousarray(K, np.float64).reshape(-1), d, len(d),
                             nk.ctypes.data if nk is not None else None, dst, w, xy, fr)
    if rc:
        raise ValueError("singular new camera matrix")
    return dst, xy, fr


THE_RNG_SEED = 0xFFFFFFFF  # cv::theRNG() of a fresh thread (RNG() state)


def flann_knn(dq, dt, k=2, trees=5, checks=50, rng_state=THE_RNG_SEED):
    """FlannBasedMatcher(KDTREE, trees).knnMatch(dq, dt, k) with search checks
    (flann.cpp): (train_idx int32[nq, k], squared distances float32[nq, k],
    the theRNG state after the call)."""
    dq = np.ascontiguousarray(dq, np.float32)
    dt = np.ascontiguousarray(dt, np.float32)
    nq, dim = dq.shape
    idx = np.zeros((max(nq, 1), k), np.int32)
    dist = np.zeros((max(nq, 1), k), np.float32)
    st = ctypes.c_uint64(rng_state)
    rc = lib().ora_flann_knn(dq.reshape(-1) if nq else np.zeros(dim, np.float32), nq, dt.reshape(-1), len(dt), dim,
                             k, trees, checks, ctypes.byref(st), idx, dist)
    if rc:
        raise ValueError("flann_knn: bad arguments (k must not exceed the train set)")
    return idx[:nq], dist[:nq], st.value


def flann_rng_after(state, train_sizes, trees=5):
    n = np.ascontiguousarray(train_sizes, np.int32)
    return int(lib().ora_flann_rng_after(state, n, len(n), trees))
