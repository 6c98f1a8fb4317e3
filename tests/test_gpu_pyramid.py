"""ORB's image pyramid on the device (OpenCV 4.x: resize INTER_LINEAR_EXACT from
the previous level, orb.cpp computeKeyPoints' buildPyramid), every level bit
for bit against the oracle (oracle/orb.cpp): resize_level_lds_kernel (a 256 x 32 tile per
workgroup from a staged source window; rs_lane / rs_word), and for level pairs
whose size ratio exceeds 1.25 resize_level_kernel.  Noise frames touch every pixel's arithmetic; odd sizes
leave partial tiles at the right and bottom edges; 9 frames run the
XCD-grouped block order (>= 8 frames)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W,H,F", [(640, 480, 2), (1280, 720, 9), (1920, 1080, 2), (1067, 601, 3), (37, 29, 2),
                                   (333, 1001, 2), (4095, 97, 1), (96, 2000, 1)])
def test_pyramid_levels_bit_exact(gpu_ctx, oracle_mod, W, H, F):
    import torch
    from droplet_visual_odometry_amd.stream import FrameStream
    rng = np.random.default_rng(W * 7 + H)
    frames = rng.integers(0, 256, (F, H, W)).astype(np.uint8)
    frames[0, : H // 2] = np.clip(np.add.outer(np.arange(H // 2), np.arange(W)) % 256, 0, 255).astype(np.uint8)
    K = np.array([[W, 0, W / 2], [0, W, H / 2], [0, 0, 1.0]])
    fs = FrameStream(W, H, K, nfeatures=500, max_frames=F, ctx=gpu_ctx)
    dev = torch.from_numpy(frames).cuda()
    fs.process(dev)
    fs.sync()
    for f in range(F):
        want = oracle_mod.pyramid(frames[f])
        for l in range(1, 8):
            np.testing.assert_array_equal(fs.pyramid(f, l), want[l], err_msg=f"frame {f} level {l}")
    fs.close()
