"""Ground-truth marker corner input for the marker-scaled pose tail (SURVEY.md
§8f rank 3).

The reference harness reads STag detections (`stag_ros` StagMarkers messages)
and hands the corners of the first marker to
`VisualOdometry.visual_odometry_calculations` as the `*_marker_corners`
arguments (`trajectory_evaluation_dual_process.py:123-124,181-185,213-237`
through `traj_eval_ground_truth.py:303-311`).  `get_stagmarker_keypoints` is
that extraction, same input and output: `markers[0].corners` (objects with
`.x`, `.y`) -> float64 [K, 2] in pixel coordinates, in message order (the
reference does not sort).  Messages are duck-typed, so rosbag messages,
`types.SimpleNamespace` objects or anything with the same attributes work
without ROS installed.

`marker_corner_batch` packs a stream of such readings (or [K, 2] arrays) into
the float64 [F, K, 2] tensor that `FrameStream.pose_tail` takes for a batch of
F frames: pair i uses rows i and i + 1 (`corners[:-1]`, `corners[1:]`), the
device form of the harness's `stagmarker_corners_list[-2]`, `[-1]`
(dual:236-237).  The scale factor only reads corners 0 and 1 (v3:269-276), so
every frame needs the same K >= 2.
"""
from __future__ import annotations

from typing import Iterable

import numpy as np


def get_stagmarker_keypoints(marker_reading) -> np.ndarray:
    """Corners of the first marker of a StagMarkers reading as float64 [K, 2]
    (traj_eval_ground_truth.py:303-311; IndexError on a reading without
    markers, as there)."""
    markers = marker_reading.markers
    corner_array = []
    for corner in markers[0].corners:
        corner_array.append([corner.x, corner.y])
    return np.array(corner_array, dtype=np.float64)


def _as_corners(item) -> np.ndarray:
    if hasattr(item, "markers"):
        return get_stagmarker_keypoints(item)
    a = np.asarray(item, dtype=np.float64)
    if a.ndim != 2 or a.shape[1] != 2:
        raise ValueError(f"marker corners must be [K, 2], got shape {a.shape}")
    return a


def marker_corner_batch(readings: Iterable, device=None):
    """Stack F readings (StagMarkers-like messages or [K, 2] arrays) into a
    float64 [F, K, 2] array, or a torch tensor on `device` when given (the
    pose-tail input of FrameStream)."""
    arrs = [_as_corners(r) for r in readings]
    if not arrs:
        raise ValueError("no marker readings")
    k = arrs[0].shape[0]
    if k < 2:
        raise ValueError("the scale factor needs at least 2 marker corners (v3:269-276)")
    for i, a in enumerate(arrs):
        if a.shape != (k, 2):
            raise ValueError(f"reading {i} has {a.shape[0]} corners, expected {k} like reading 0")
    out = np.ascontiguousarray(np.stack(arrs))
    if device is None:
        return out
    import torch
    return torch.from_numpy(out).to(device)
