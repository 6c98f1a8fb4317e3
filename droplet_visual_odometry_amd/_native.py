"""ctypes binding of libdvo_hip.so (include/dvo.h).

There is no CPU fallback: if the HIP library is missing or no GPU is visible,
every compute entry point raises.  PyTorch is imported first when available so
the library binds to the same HIP runtime as torch (one runtime, one device
address space; see build.py).
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

try:  # load torch's HIP runtime first (shared runtime); torch is plumbing only
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is always present in this image
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
# DVO_LIB_PATH: an experiment build of the same sources (tools/ A/B runs); default the in-tree product build
_DEFAULT_LIB = os.path.join(HERE, "lib", "libdvo_hip.so")
LIB_PATH = os.environ.get("DVO_LIB_PATH") or _DEFAULT_LIB

DVO_OK = 0
DVO_EINVAL = -1
DVO_ENOFEAT = -2
DVO_EFEWPTS = -3
DVO_EHIP = -4
DVO_ECAP = -5
DVO_ENOMODEL = -6
DVO_NSTAGES = 9
STAGE_NAMES = ["pyramid", "blur", "fast", "select_harris", "describe", "match", "ransac", "recover_pose",
               "pose_tail"]

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
DMATCH_DTYPE = np.dtype([("queryIdx", "<i4"), ("trainIdx", "<i4"), ("imgIdx", "<i4"), ("distance", "<f4")])
PAIR_RECORD_DTYPE = np.dtype([("R", "<f8", (9,)), ("t", "<f8", (3,)), ("E", "<f8", (9,)),
                              ("n_kp_prev", "<i4"), ("n_kp_cur", "<i4"), ("n_matches", "<i4"),
                              ("n_inliers", "<i4"), ("n_good", "<i4"), ("ransac_iters", "<i4"),
                              ("status", "<i4"), ("n_models", "<i4"), ("n_hypotheses", "<i4"), ("pad0", "<i4"),
                              ("reserved", "<f8", (6,))])
assert PAIR_RECORD_DTYPE.itemsize == 256


class DVOError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"dvo error {code}: {msg}")
        self.code = code


class OrbParams(ctypes.Structure):
    _fields_ = [("nfeatures", ctypes.c_int32), ("scale_factor", ctypes.c_float), ("nlevels", ctypes.c_int32),
                ("edge_threshold", ctypes.c_int32), ("first_level", ctypes.c_int32), ("wta_k", ctypes.c_int32),
                ("score_type", ctypes.c_int32), ("patch_size", ctypes.c_int32), ("fast_threshold", ctypes.c_int32),
                ("opencv_semantics", ctypes.c_int32)]


class StreamConfig(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("max_frames", ctypes.c_int32),
                ("orb", OrbParams), ("K", ctypes.c_double * 9), ("prob", ctypes.c_double),
                ("threshold", ctypes.c_double), ("max_iters", ctypes.c_int32), ("cross_check", ctypes.c_int32),
                ("dist_thresh", ctypes.c_double)]


# OpenCV semantics of the ORB path (include/dvo.h DVO_OPENCV_*): "4.x" (default) or "3.2"
OPENCV_SEMANTICS = {"4.x": 0, "3.2": 1}


def opencv_semantics(v) -> int:
    if isinstance(v, str):
        if v not in OPENCV_SEMANTICS:
            raise ValueError(f"opencv semantics must be one of {sorted(OPENCV_SEMANTICS)}")
        return OPENCV_SEMANTICS[v]
    if int(v) not in OPENCV_SEMANTICS.values():
        raise ValueError(f"opencv semantics must be one of {sorted(OPENCV_SEMANTICS)}")
    return int(v)


def orb_params(nfeatures=500, scale_factor=1.2, nlevels=8, edge_threshold=31, first_level=0, wta_k=2,
               score_type=0, patch_size=31, fast_threshold=20, opencv="4.x") -> OrbParams:
    return OrbParams(int(nfeatures), float(np.float32(scale_factor)), int(nlevels), int(edge_threshold),
                     int(first_level), int(wta_k), int(score_type), int(patch_size), int(fast_threshold),
                     opencv_semantics(opencv))


_vp = ctypes.c_void_p
_ip = ctypes.POINTER(ctypes.c_int)
_c = ctypes.c_int
_d = ctypes.c_double
_i64 = ctypes.c_int64

_SIGNATURES = {
    "dvo_version": ([], _c),
    "dvo_build_id": ([], ctypes.c_char_p),
    "dvo_ctx_create": ([ctypes.POINTER(_vp), _c], _c),
    "dvo_ctx_destroy": ([_vp], None),
    "dvo_last_error": ([_vp], ctypes.c_char_p),
    "dvo_orb_detect_and_compute": ([_vp, ctypes.POINTER(OrbParams), _vp, _c, _c, _c, _vp, _vp, _c, _ip], _c),
    "dvo_bf_match_hamming": ([_vp, _vp, _c, _vp, _c, _c, _vp, _c, _ip], _c),
    "dvo_bf_knn_float": ([_vp, _vp, _c, _vp, _c, _c, _c, _c, _vp, _vp], _c),
    "dvo_flann_knn": ([_vp, _vp, _c, _vp, _c, _c, _c, _c, _c, ctypes.POINTER(ctypes.c_uint64), _vp, _vp], _c),
    "dvo_sift_detect_and_compute": ([_vp, _vp, _c, _c, _c, _vp, _vp, _c, _ip], _c),
    "dvo_surf_detect_and_compute": ([_vp, _vp, _c, _c, _c, ctypes.c_double, _vp, _vp, _c, _ip], _c),
    "dvo_find_essential_mat": ([_vp, _vp, _vp, _c, _vp, _d, _d, _c, _vp, _ip, _vp], _c),
    "dvo_recover_pose": ([_vp, _vp, _c, _vp, _vp, _c, _vp, _d, _vp, _vp, _vp, _vp, _ip], _c),
    "dvo_triangulate_points": ([_vp, _vp, _vp, _vp, _vp, _c, _vp], _c),
    "dvo_stream_create": ([_vp, ctypes.POINTER(StreamConfig), ctypes.POINTER(_vp)], _c),
    "dvo_stream_destroy": ([_vp], None),
    "dvo_stream_process": ([_vp, _vp, _c, _i64, _c, _vp], _c),
    "dvo_stream_process_pairs": ([_vp, _vp, _c, _i64, _c, _vp], _c),
    "dvo_pipeline_depth": ([], _c),
    "dvo_stream_submit": ([_vp, _vp, _c, _i64, _c, _vp], _c),
    "dvo_stream_submit_pairs": ([_vp, _vp, _c, _i64, _c, _vp], _c),
    "dvo_stream_drain": ([_vp], _c),
    "dvo_stream_retired": ([_vp, ctypes.POINTER(_vp), _ip, _c], _c),
    "dvo_stream_pose_tail_batch": ([_vp, _vp, _c, _vp, _vp, _c, _d, _vp, _vp], _c),
    "dvo_stream_pair": ([_vp, _vp, _vp, _c, _c, _vp], _c),
    "dvo_stream_sync": ([_vp], _c),
    "dvo_stream_hip_stream": ([_vp], _vp),
    "dvo_stream_set_profiling": ([_vp, _c], _c),
    "dvo_stream_reset_pose": ([_vp, _vp, _vp], _c),
    "dvo_get_optimal_new_camera_matrix": ([_vp, _vp, _c, _c, _c, _d, _c, _c, _vp], _c),
    "dvo_undistort_create": ([_vp, _vp, _vp, _c, _vp, _c, _c, _vp], _c),
    "dvo_undistort_destroy": ([_vp], None),
    "dvo_undistort_apply": ([_vp, _vp, _c, ctypes.c_int64, _c, _vp, ctypes.c_int64, _c, _vp], _c),
    "dvo_undistort_image": ([_vp, _vp, _c, _vp, _c], _c),
    "dvo_undistort_get_map": ([_vp, _vp, _vp], _c),
    "dvo_stream_process_undistorted": ([_vp, _vp, _vp, _c, _i64, _c, _vp], _c),
    "dvo_stream_share_pose": ([_vp, _vp], _c),
    "dvo_stream_pose_tail": ([_vp, _vp, _vp, _c, _d, _vp, _vp], _c),
    "dvo_pose_tail_records": ([_vp, _vp, _c, _vp, _vp, _vp, _c, _d, _vp, _vp, _vp, _vp], _c),
    "dvo_pose_chain": ([_vp, _vp, _c, _vp, _vp, _vp], _c),
    "dvo_pose_chain_host": ([_vp, _c, _vp, _vp], _c),
    "dvo_pose_rel_range": ([_vp, _vp, _c, _c, _c, _vp, _vp, _vp, _c, _d, _vp, _vp, _vp], _c),
    "dvo_stream_stage_times": ([_vp, _vp, _ip], _c),
    "dvo_stream_get_features": ([_vp, _c, _vp, _vp, _c, _ip], _c),
    "dvo_stream_get_matches": ([_vp, _c, _vp, _c, _ip], _c),
    "dvo_stream_get_pyramid": ([_vp, _c, _c, _c, _vp, _c], _c),
    "dvo_test_retain_best": ([_vp, _vp, _c, _c, _c, _c, _vp, _ip], _c),
    "dvo_test_update_num_iters": ([_vp, _d, _vp, _c, _c, _c, _vp], _c),
    "dvo_test_five_point": ([_vp, _vp, _vp, _vp, _ip], _c),
    "dvo_test_sampson": ([_vp, _vp, _vp, _c, ctypes.c_float, _vp, _vp], _c),
    "dvo_test_ransac_subsets": ([_vp, _c, _c, _vp], _c),
    "dvo_test_ransac_replay": ([_vp, _vp, _vp, _c, _c, _d, _c, _vp], _c),
}

_lib = None
_lock = threading.Lock()


def load_library(path: str = LIB_PATH):
    """Load libdvo_hip.so; raises if it is absent (no CPU fallback exists)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise ImportError(f"{path} is missing: build it with `python -m droplet_visual_odometry_amd.build` "
                              "(hipcc, gfx950). droplet_visual_odometry_amd has no CPU fallback.")
        L = ctypes.CDLL(path)
        for name, (args, res) in _SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        if path == _DEFAULT_LIB and os.path.isdir(os.path.join(HERE, "csrc")):
            from .build import source_hash
            want, got = source_hash(), L.dvo_build_id().decode()
            if got != want:
                raise ImportError(f"{path} was built from other sources (build id {got}, sources {want}): "
                                  "rebuild it with `python -m droplet_visual_odometry_amd.build`")
        _lib = L
        return L


def exported_symbols():
    return list(_SIGNATURES)


def ptr(a) -> int:
    """Raw pointer of a numpy array or torch tensor (None -> 0)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()


class Context:
    """One dvo_ctx (device, HIP stream, scratch).  Not thread-safe; one per host thread."""

    _tls = threading.local()

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = _vp()
        rc = self.lib.dvo_ctx_create(ctypes.byref(h), int(device))
        if rc != DVO_OK:
            raise DVOError(rc, f"dvo_ctx_create(device={device}) failed: no usable HIP device")
        self.h = h
        self.device = device

    @classmethod
    def default(cls, device: int = 0) -> "Context":
        ctxs = getattr(cls._tls, "ctxs", None)
        if ctxs is None:
            ctxs = cls._tls.ctxs = {}
        if device not in ctxs:
            ctxs[device] = cls(device)
        return ctxs[device]

    def check(self, rc):
        if rc != DVO_OK:
            msg = self.lib.dvo_last_error(self.h)
            raise DVOError(rc, msg.decode() if msg else "")
        return rc

    def close(self):
        if getattr(self, "h", None):
            self.lib.dvo_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
