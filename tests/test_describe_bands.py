"""describe_kernel blurs only the pixels a rotated rBRIEF pattern point can
round to (csrc/orb.hip kDBRows / kDBBase / kDBHalfW; orb.cpp computeOrbDescriptors,
reached from visual_odometry_v3.py:373).  Checked here on the host, from the
constants in orb.hip: every (dy, dx) that cvRound of the float32 rotation of a
pattern point reaches, over a fine angle sweep and by the closed-form bound,
lies in a band row whose word range (for every 4-byte alignment of the
keypoint) holds it, with a halo word on each side, inside the 13 raw words."""
import math
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _consts():
    src = open(os.path.join(ROOT, "droplet_visual_odometry_amd", "csrc", "orb.hip")).read()
    block = src[src.index("constexpr int kDBRows"):]
    rows = int(re.search(r"kDBRows = (\d+), kDBSeg = (\d+)", block).group(1))
    seg = int(re.search(r"kDBRows = (\d+), kDBSeg = (\d+)", block).group(2))
    row0 = int(re.search(r"kDBRow0 = (\d+)", block).group(1))
    base = [int(v) for v in re.search(r"kDBBase\[kDBSeg \+ 1\] = \{([^}]*)\}", block).group(1).split(",")]
    halfw = [int(v) for v in re.search(r"kDBHalfW\[kDBSeg\] = \{([^}]*)\}", block).group(1).split(",")]
    return rows, seg, row0, base, halfw


def _pattern():
    txt = open(os.path.join(ROOT, "data", "orb_bit_pattern_31.inc")).read()
    body = "\n".join(l for l in txt.splitlines() if not l.lstrip().startswith("//"))
    return np.array([int(v) for v in re.findall(r"-?\d+", body)], np.int32).reshape(-1, 2)


def test_bands_cover_every_sampled_pixel():
    rows, seg, row0, base, halfw = _consts()
    assert base[-1] <= 64
    P = _pattern()
    assert len(P) == 512
    ang = np.linspace(0, 2 * np.pi, 100001)
    ca, sa = np.cos(ang).astype(np.float32), np.sin(ang).astype(np.float32)
    px, py = P[:, 0].astype(np.float32)[None], P[:, 1].astype(np.float32)[None]
    xi = np.rint((px * ca[:, None] - py * sa[:, None]).astype(np.float32)).astype(int)
    yi = np.rint((px * sa[:, None] + py * ca[:, None]).astype(np.float32)).astype(int)
    r = float(np.hypot(P[:, 0], P[:, 1]).max()) + 1e-3
    need = {}
    for dy in range(-19, 20):  # sweep extents and the closed-form bound, whichever is larger
        m = yi == dy
        sweep = int(np.abs(xi[m]).max()) if m.any() else -1
        a = abs(dy)
        if a > r + 0.5:
            bound = -1
        else:
            lim = r if a == 0 else math.sqrt(max(r * r - (a - 0.5) ** 2, 0.0))
            bound = math.floor(lim + 0.5) if a - 0.5 <= r else -1
        assert sweep <= bound
        if bound >= 0:
            need[dy] = bound
    for dy, w in need.items():
        i = dy + 19  # patch row (row 0 <-> dy = -19)
        s = (i - row0) // rows
        assert 0 <= s < seg and row0 + rows * s <= i < row0 + rows * (s + 1), dy
        assert w <= halfw[s], (dy, w, halfw[s])
        nw = base[s + 1] - base[s]
        for o in range(19, 23):  # cx - a0: a0 = (cx - 19) & ~3
            wlo = (o - halfw[s]) >> 2
            lanes = [min(wlo + k, 12) for k in range(nw)]
            store = lanes[1:nw - 1]  # the band's halo lanes do not store
            for dx in range(-w, w + 1):
                word = ((o + dx) >> 2) + 1  # raw word of [a0 - 4, a0 + 48)
                assert 1 <= word <= 11 and word in store, (dy, dx, o, word, store)
            assert wlo + nw - 1 <= 12
