"""ORB pyramid geometry (host-side shape logic, mirrored by csrc/api.cpp make_plan).

orb.cpp detectAndCompute: level l has scale s_l = (float)pow(double(1.2f), l)
and size cvRound(W * (1.0f / s_l)) x cvRound(H * (1.0f / s_l)) in float
arithmetic; computeKeyPoints splits nfeatures over the levels geometrically.
"""
from __future__ import annotations

import numpy as np

SCALE_FACTOR = float(np.float32(1.2))  # ORB_Impl::scaleFactor = double(1.2f)


def level_scale(level: int) -> np.float32:
    return np.float32(SCALE_FACTOR ** level)


def level_sizes(w: int, h: int, nlevels: int = 8):
    out = []
    for l in range(nlevels):
        inv = np.float32(1.0) / level_scale(l)
        if l == 0:
            out.append((w, h))
        else:
            out.append((int(np.rint(np.float32(w) * inv)), int(np.rint(np.float32(h) * inv))))
    return out


def features_per_level(nfeatures: int, nlevels: int = 8):
    factor = np.float32(1.0 / SCALE_FACTOR)
    nd = np.float32(nfeatures) * (np.float32(1) - factor) / (np.float32(1) - np.float32(float(factor) ** nlevels))
    out, s = [], 0
    for _ in range(nlevels - 1):
        v = int(np.rint(nd))
        out.append(v)
        s += v
        nd = np.float32(nd * factor)
    out.append(max(nfeatures - s, 0))
    return out


def algorithmic_bytes_per_frame(w: int, h: int, nfeatures: int, n_matches: float | None = None) -> float:
    """B = 2 * sum_l W_l H_l + 64 N + 16 M (M = N/2 nominal)."""
    px = sum(a * b for a, b in level_sizes(w, h))
    m = nfeatures / 2 if n_matches is None else n_matches
    return 2.0 * px + 64.0 * nfeatures + 16.0 * m
