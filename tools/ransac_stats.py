"""Distribution of RANSAC iterations over one batch of the bench stream (pairs
needing more than r hypotheses, for choosing the round sizes).

usage: python tools/ransac_stats.py [--batch 1024] [--width 1280 --height 720 --nfeatures 2000]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from droplet_visual_odometry_amd._native import Context  # noqa: E402
from droplet_visual_odometry_amd.stream import FrameStream  # noqa: E402
from droplet_visual_odometry_amd.synth import SceneStream  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--nfeatures", type=int, default=2000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    scene = SceneStream(a.width, a.height, device=str(dev))
    frames = torch.stack([scene.render(i) for i in range(a.batch + 1)]).contiguous()
    fs = FrameStream(a.width, a.height, scene.K, nfeatures=a.nfeatures, max_frames=a.batch + 1, ctx=Context(0))
    rec = fs.process(frames)
    fs.sync()
    r = FrameStream.records_numpy(rec, a.batch)
    it, hy = r["ransac_iters"], r["n_hypotheses"]
    print("iterations: mean %.1f  percentiles 10/50/90/99/max: %s" % (it.mean(), np.percentile(it, [10, 50, 90, 99, 100])))
    print("hypotheses solved: mean %.1f" % hy.mean())
    for t in (64, 96, 128, 160, 192, 256, 384, 512):
        print(f"  pairs needing > {t:4d}: {int((it > t).sum()):5d}   hypotheses wasted if round 1 = {t}: "
              f"{float(np.maximum(0, t - it).mean()):.1f} per pair")


if __name__ == "__main__":
    main()
