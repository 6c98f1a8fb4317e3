"""cProfile of the drop-in per-pair surface (VisualOdometry.visual_odometry_calculations)
on the GPU box: where a synchronous pair's wall time goes (host Python, ctypes calls).
Usage: python tools/profile_dropin.py [W H N]"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from droplet_visual_odometry_amd.synth import SceneStream
    W, H, N = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (1280, 720, 2000)
    st = SceneStream(W, H, device="cuda")
    pool = torch.stack([st.render(i) for i in range(24)])
    import numpy as np
    corners = torch.tensor(np.stack([st.marker_corners(i) for i in range(24)]))
    print(bench.dropin_rate(pool, corners, st.K, N, 2.0, n_frames=24))
    pr = cProfile.Profile()
    pr.enable()
    r = bench.dropin_rate(pool, corners, st.K, N, 3.0, n_frames=24)
    pr.disable()
    print(r)
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
