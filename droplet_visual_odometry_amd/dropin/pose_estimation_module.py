"""Drop-in replacement for the reference's scripts/pose_estimation_module.py.

Same functions and outputs (pem:15-184).  ROS `tf` (pem:8) is replaced by the
numpy restatement in droplet_visual_odometry_amd.transformations, exposed as
the module attribute `tf` with both spellings the reference uses
(`tf.quaternion_matrix`, `tf.transformations.euler_from_quaternion`), so the
module imports without a ROS installation.  Plotting helpers import
matplotlib lazily.
"""
from __future__ import annotations

import types

import numpy as np

from droplet_visual_odometry_amd import transformations as _tr

tf = types.SimpleNamespace(transformations=_tr, quaternion_matrix=_tr.quaternion_matrix,
                           euler_from_quaternion=_tr.euler_from_quaternion,
                           euler_from_matrix=_tr.euler_from_matrix)


def transformation_from_translation_quaternion(translation, quaternion):
    """4x4 from a translation and an (x, y, z, w) quaternion (pem:15-23)."""
    T = np.eye(4)
    T[:3, :3] = tf.quaternion_matrix(quaternion)[:3, :3]
    T[:3, 3] = translation
    return T


def translation_from_transformation_matrix(transformation_matrix):
    """[tx, ty, tz] of a 4x4 (pem:26-28)."""
    return [transformation_matrix[0, 3], transformation_matrix[1, 3], transformation_matrix[2, 3]]


def rotation_matrix_to_quaternion(rotation_matrix):
    """Trace-branch quaternion [x, y, z, w], not renormalised (pem:31-57)."""
    R = rotation_matrix
    trace = np.trace(R)
    if trace > 0:
        S = np.sqrt(trace + 1.0) * 2.0
        return [(R[2, 1] - R[1, 2]) / S, (R[0, 2] - R[2, 0]) / S, (R[1, 0] - R[0, 1]) / S, 0.25 * S]
    if (R[0, 0] > R[1, 1]) and (R[0, 0] > R[2, 2]):
        S = np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2.0
        return [0.25 * S, (R[0, 1] + R[1, 0]) / S, (R[0, 2] + R[2, 0]) / S, (R[2, 1] - R[1, 2]) / S]
    if R[1, 1] > R[2, 2]:
        S = np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2.0
        return [(R[0, 1] + R[1, 0]) / S, 0.25 * S, (R[1, 2] + R[2, 1]) / S, (R[0, 2] - R[2, 0]) / S]
    S = np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2.0
    return [(R[0, 2] + R[2, 0]) / S, (R[1, 2] + R[2, 1]) / S, 0.25 * S, (R[1, 0] - R[0, 1]) / S]


def quaternion_from_transformation_matrix(transformation_matrix):
    return rotation_matrix_to_quaternion(transformation_matrix[:3, :3])


def get_marker_to_marker_transformation(previous_cTm_transform, current_cTm_transform):
    return np.matmul(np.linalg.inv(previous_cTm_transform), current_cTm_transform)


def get_camera_to_camera_transformation(previous_cTm_transform, current_cTm_transform):
    return np.matmul(previous_cTm_transform, np.linalg.inv(current_cTm_transform))


def _tum_line(timestamp, translation, quaternion):
    vals = [timestamp, translation[0], translation[1], translation[2], quaternion[0], quaternion[1], quaternion[2],
            quaternion[3]]
    return " ".join(str(v) for v in vals) + " " + "\n"


def write_to_output_file(output_file_path, timestamp, translation, quaternion):
    """Append `ts tx ty tz qx qy qz qw ` + newline (pem:80-86; note the trailing space)."""
    with open(output_file_path, "a") as fh:
        fh.write(_tum_line(timestamp, translation, quaternion))


def clear_txt_file_contents(file_path):
    with open(file_path, "w") as fh:
        fh.truncate()


def get_velocity_between_timestamps(relative_position_change, previous_timestamp, current_timestamp):
    """t / dt and R / dt packed into a 4x4 (pem:94-111, element-wise as written)."""
    dt = current_timestamp - previous_timestamp
    v = np.eye(4)
    v[:3, :3] = relative_position_change[:3, :3] / dt
    v[:3, 3] = np.array([relative_position_change[0, 3], relative_position_change[1, 3],
                         relative_position_change[2, 3]]) / dt
    return v


def get_gt_vo_difference(gt_file_path, vo_file_path):
    gt = np.genfromtxt(gt_file_path)
    vo = np.genfromtxt(vo_file_path)
    for i in range(gt.shape[0] - 1):
        g = np.array(tf.transformations.euler_from_quaternion(tuple(gt[i, 4:8])))
        v = np.array(tf.transformations.euler_from_quaternion(tuple(vo[i, 4:8])))
        return v - g


def write_gt_vo_difference_to_file(gt_file_path, vo_file_path, output_file_path):
    gt = np.genfromtxt(gt_file_path)
    vo = np.genfromtxt(vo_file_path)
    with open(output_file_path, "w") as fh:
        for i in range(gt.shape[0] - 1):
            g = np.array(tf.transformations.euler_from_quaternion(tuple(gt[i, 4:8])))
            v = np.array(tf.transformations.euler_from_quaternion(tuple(vo[i, 4:8])))
            fh.write("at timestamp {} the gt vo euler angle difference is {} \n".format(gt[i, 0], v - g))


def append_transformation_to_file(transformation_matrix, file_path):
    with open(file_path, "a") as fh:
        for row in transformation_matrix:
            fh.write(" ".join(str(value) for value in row) + "\n")


def compute_gt_vo_translation_difference(gt_file_path, vo_file_path):
    gt = np.genfromtxt(gt_file_path)
    vo = np.genfromtxt(vo_file_path)
    d = np.array([vo[1], vo[2], vo[3]]) - np.array([gt[1], gt[2], gt[3]])
    return [d[0], d[1], d[2]]


def visualize_gt_vo_translation_difference(translation_difference, plot_output_path):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig = plt.figure(figsize=(5, 5))
    ax = fig.add_subplot(111, projection="3d")
    d = translation_difference
    ax.scatter(d[0], d[1], d[2], c="r", marker="o")
    ax.set_xlabel("X")
    ax.set_ylabel("Y")
    ax.set_zlabel("Z")
    ax.set_title("Translation Difference Visualization")
    fig.savefig(plot_output_path, format="jpg", dpi=100)
    plt.close(fig)
