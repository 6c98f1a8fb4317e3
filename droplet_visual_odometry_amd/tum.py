"""Batch pose-stream writer.

The reference's trajectory harness logs, per processed frame, three TUM files
(trajectory_evaluation_dual_process.py:254-290, via pose_estimation_module
pem:26-111): the absolute VO pose T_robot (vo_absolute_position_list), the
relative transform T_prev->cur (vo_camera_to_camera_list) and the "velocity"
transform (pem.get_velocity_between_timestamps: t/dt and R/dt element-wise).
Each line is `ts tx ty tz qx qy qz qw ` + newline, with the trace-branch
quaternion (x, y, z, w) of pem.rotation_matrix_to_quaternion, not renormalised.

PoseStreamWriter takes whole batches (the device T_rel / T_abs of
FrameStream.pose_tail, or the host chain after dist.gather_records) and writes
the same text the harness writes one pose at a time.  Floats are formatted
with Python 3 `str()` (the reference ran Python 2, whose str() keeps 12
significant digits; use fmt=lambda v: "%.12g" % v to reproduce that).
"""
from __future__ import annotations

import numpy as np

from droplet_visual_odometry_amd.dropin import pose_estimation_module as pem


def tum_line(timestamp, T, fmt=str) -> str:
    """One harness line for a 4x4 transform (dual:275-290)."""
    t = pem.translation_from_transformation_matrix(T)
    q = pem.quaternion_from_transformation_matrix(T)
    vals = [timestamp, t[0], t[1], t[2], q[0], q[1], q[2], q[3]]
    return " ".join(fmt(v) for v in vals) + " " + "\n"


class PoseStreamWriter:
    """Appends the harness's three VO logs for consecutive batches.

    paths: dict with keys 'absolute', 'relative', 'velocity' (any subset)."""

    def __init__(self, paths: dict, start_timestamp=None, start_pose=None, fmt=str, truncate=True):
        self.paths = dict(paths)
        self.fmt = fmt
        self.prev_ts = start_timestamp
        if truncate:
            for p in self.paths.values():
                pem.clear_txt_file_contents(p)
        if start_timestamp is not None and start_pose is not None and "absolute" in self.paths:
            # dual:197-198: the starting pose is the first absolute entry
            with open(self.paths["absolute"], "a") as fh:
                fh.write(tum_line(start_timestamp, np.asarray(start_pose, np.float64), fmt))

    def write_batch(self, timestamps, T_abs, T_rel):
        """timestamps [n] of the batch's current frames; T_abs / T_rel [n, 4, 4]
        (numpy or torch, any device)."""
        T_abs = _np(T_abs)
        T_rel = _np(T_rel)
        ts = list(timestamps)
        if not (len(ts) == len(T_abs) == len(T_rel)):
            raise ValueError("timestamps, T_abs and T_rel must have the same length")
        out = {k: [] for k in self.paths}
        for i, t in enumerate(ts):
            if "absolute" in out:
                out["absolute"].append(tum_line(t, T_abs[i], self.fmt))
            if "relative" in out:
                out["relative"].append(tum_line(t, T_rel[i], self.fmt))
            if "velocity" in out and self.prev_ts is not None:
                v = pem.get_velocity_between_timestamps(T_rel[i], self.prev_ts, t)
                out["velocity"].append(tum_line(t, v, self.fmt))
            self.prev_ts = t
        for k, lines in out.items():
            with open(self.paths[k], "a") as fh:
                fh.write("".join(lines))


def _np(x):
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x, np.float64)
