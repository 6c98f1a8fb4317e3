"""Ground-truth corner input (traj_eval_ground_truth.py:303-311) and its batch
packing for the device pose tail: CPU tests with duck-typed StagMarkers
messages (no ROS)."""
import os
import sys
from types import SimpleNamespace as NS

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "droplet_visual_odometry_amd", "dropin"))
import marker_corners as mc  # noqa: E402


def reading(pts, extra_markers=()):
    first = NS(id=7, corners=[NS(x=float(x), y=float(y), z=0.0) for x, y in pts])
    return NS(markers=[first, *extra_markers])


def test_first_marker_corners_in_message_order():
    pts = [(310.5, 200.25), (350.0, 201.0), (349.5, 240.75), (309.0, 239.5)]
    other = NS(id=3, corners=[NS(x=1.0, y=2.0)] * 4)
    a = mc.get_stagmarker_keypoints(reading(pts, [other]))
    assert a.dtype == np.float64 and a.shape == (4, 2)
    np.testing.assert_array_equal(a, np.array(pts))


def test_no_marker_raises_like_the_reference():
    with pytest.raises(IndexError):
        mc.get_stagmarker_keypoints(NS(markers=[]))


def test_empty_corner_list_matches_reference_shape():
    assert mc.get_stagmarker_keypoints(reading([])).shape == (0,)


def test_batch_stacks_messages_and_arrays():
    rng = np.random.default_rng(5)
    frames = [rng.uniform(0, 640, (4, 2)) for _ in range(5)]
    mixed = [reading(f) if i % 2 else f for i, f in enumerate(frames)]
    b = mc.marker_corner_batch(mixed)
    assert b.shape == (5, 4, 2) and b.dtype == np.float64 and b.flags.c_contiguous
    np.testing.assert_array_equal(b, np.stack(frames))
    # pair i of a batch uses frames i and i + 1, as the harness's corners_list[-2], [-1]
    np.testing.assert_array_equal(b[:-1][2], frames[2])
    np.testing.assert_array_equal(b[1:][2], frames[3])


def test_batch_rejects_inconsistent_or_short_readings():
    with pytest.raises(ValueError):
        mc.marker_corner_batch([np.zeros((4, 2)), np.zeros((3, 2))])
    with pytest.raises(ValueError):
        mc.marker_corner_batch([np.zeros((1, 2))])
    with pytest.raises(ValueError):
        mc.marker_corner_batch([np.zeros((4, 3))])
    with pytest.raises(ValueError):
        mc.marker_corner_batch([])


def test_batch_to_torch_tensor_on_cpu():
    torch = pytest.importorskip("torch")
    b = mc.marker_corner_batch([np.ones((4, 2)), np.zeros((4, 2))], device="cpu")
    assert isinstance(b, torch.Tensor) and b.dtype == torch.float64 and tuple(b.shape) == (2, 4, 2)
