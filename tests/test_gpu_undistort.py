"""GPU undistortion (dvo_undistort_*, cv.undistort of visual_odometry_v3.py:120)
vs the oracle restatement: remap table and remapped image bit-exact, for the
reference's two calibration files, zero distortion and a rational model."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = [
    (np.zeros(5), (640, 480)),
    (np.array([0.142541, -0.248887, -0.005254, -0.005417, 0.0]), (640, 480)),      # rosbot_calibration.yaml:22
    (np.array([-0.296079, 0.099771, 0.000222, 0.000109, 0.0]), (1440, 1080)),      # camera_calibration.yaml:22
    (np.array([0.1, -0.2, 0.001, -0.002, 0.05, 0.01, -0.02, 0.003]), (1280, 720)),
]


def _K(size):
    if size[0] > 640:
        return np.array([[1173.854081, 0, 747.788206], [0, 1170.565083, 574.700374], [0, 0, 1.0]])
    return np.array([[606.811009, 0, 325.199941], [0, 611.104701, 227.591593], [0, 0, 1.0]])


def _image(w, h, seed=0):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    return ((x * 7 + y * 3 + rng.integers(0, 60, (h, w))) % 256).astype(np.uint8)


@pytest.mark.parametrize("dist,size", CASES)
def test_undistort_bit_exact(gpu_ctx, oracle_mod, dist, size):
    from droplet_visual_odometry_amd import cv, ops
    w, h = size
    K = _K(size)
    newK, _ = cv.getOptimalNewCameraMatrix(K, dist, size, 1, size)
    img = _image(w, h)
    want, xy_o, fr_o = oracle_mod.undistort(img, K, dist, newK)
    u = ops.Undistorter(K, dist, newK, w, h, ctx=gpu_ctx)
    xy, fr = u.map()
    np.testing.assert_array_equal(xy, xy_o)
    np.testing.assert_array_equal(fr, fr_o)
    np.testing.assert_array_equal(u.image(img), want)
    np.testing.assert_array_equal(cv.undistort(img, K, dist, None, newK), want)
    u.close()


def test_stream_process_undistorted(gpu_ctx):
    """Undistort-then-detect in one stream call equals remapping first."""
    import torch
    from conftest import synth_frames
    from droplet_visual_odometry_amd import cv, ops
    from droplet_visual_odometry_amd.stream import FrameStream
    frames, K = synth_frames(640, 480, range(4))
    dist = np.array([0.142541, -0.248887, -0.005254, -0.005417, 0.0])
    newK, _ = cv.getOptimalNewCameraMatrix(K, dist, (640, 480), 1, (640, 480))
    u = ops.Undistorter(K, dist, newK, 640, 480, ctx=gpu_ctx)
    dev = torch.from_numpy(frames).cuda()
    und = torch.empty_like(dev)
    u.apply(dev, und)
    torch.cuda.synchronize()
    a = FrameStream(640, 480, K, nfeatures=500, max_frames=4, ctx=gpu_ctx)
    ra = a.process(und)
    b = FrameStream(640, 480, K, nfeatures=500, max_frames=4, ctx=gpu_ctx)
    rb = b.process(dev, undistort=u)
    a.sync()
    b.sync()
    np.testing.assert_array_equal(FrameStream.records_numpy(ra, 3), FrameStream.records_numpy(rb, 3))
    for fs in (a, b):
        fs.close()
    u.close()
