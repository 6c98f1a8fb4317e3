"""FAST workload statistics of the synthetic stream (CPU, numpy): the fraction
of level-0 score pixels that pass the compass pre-test, that are FAST-9
corners, and that survive a strict 3x3 NMS on a score proxy.  These set the
per-tile list lengths of fast_strip_kernel (candidates, corners, keeps).

usage: python tools/fast_stats.py [W H frame]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from droplet_visual_odometry_amd.synth import SceneStream  # noqa: E402

CY = [3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3]
CX = [0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1]


def run9(m):
    m2 = np.concatenate([m, m[:8]], 0)
    r = np.zeros(m.shape[1:], bool)
    for s in range(16):
        r |= np.all(m2[s:s + 9], 0)
    return r


def stats(img, t=20, border=30):
    img = img.astype(np.int32)
    H, W = img.shape
    y0, y1, x0, x1 = border, H - border, border, W - border
    v = img[y0:y1, x0:x1]
    circ = np.stack([img[y0 + dy:y1 + dy, x0 + dx:x1 + dx] for dx, dy in zip(CX, CY)])
    c0, c4, c8, c12 = circ[0], circ[4], circ[8], circ[12]
    comp = (np.minimum(np.maximum(c0, c8), np.maximum(c4, c12)) > v + t) | \
           (np.maximum(np.minimum(c0, c8), np.minimum(c4, c12)) < v - t)
    corner = run9(circ > v + t) | run9(circ < v - t)
    score = np.zeros(v.shape, np.int32)  # proxy: largest threshold still a corner
    for tt in range(t, 255, 4):
        ok = corner & (run9(circ > v + tt) | run9(circ < v - tt))
        if not ok.any():
            break
        score[ok] = tt
    s = np.pad(score, 1)
    nb = np.max(np.stack([s[1 + dy:1 + dy + v.shape[0], 1 + dx:1 + dx + v.shape[1]]
                          for dy in (-1, 0, 1) for dx in (-1, 0, 1) if dy or dx]), 0)
    keep = corner & (score > nb)
    return comp.mean(), corner.mean(), keep.mean()


if __name__ == "__main__":
    W, H, fr = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (1280, 720, 5)))
    img = SceneStream(W, H).render(fr).numpy()
    c, k, kp = stats(img)
    print(f"{W}x{H} frame {fr}: compass pass {100 * c:.2f}%  corners {100 * k:.2f}%  NMS keeps ~{100 * kp:.2f}% "
          f"(per 16x128 tile: {2048 * c:.0f} candidates, {2048 * k:.0f} corners, ~{2016 * kp:.0f} keeps)")
