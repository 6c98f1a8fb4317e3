"""RANSAC round schedules simulated on the CPU oracle (VERDICT 4, item 2:
hypotheses solved vs iterations used).  For each pair of the bench stream the
oracle's matched points, getSubset stream, five-point models and Sampson counts
of every hypothesis up to maxIters are computed once; any schedule of rounds is
then replayed exactly (RANSACPointSetRegistrator::run's bookkeeping), giving
the hypotheses each schedule solves and the rounds it needs.

usage: python tools/ransac_schedule_sim.py [--pairs 256] [--width 1280 --height 720 --nfeatures 2000]
       [--cache /tmp/ransac_sim.npz]"""
import argparse
import os
import sys
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

A = None


def _detect(i):
    import torch
    torch.set_num_threads(1)
    from droplet_visual_odometry_amd.synth import SceneStream
    st = SceneStream(A.width, A.height)
    img = st.render(i).numpy()
    return oracle.detect_and_compute(img, A.nfeatures), st.K


def _counts(job):
    """Per-hypothesis model counts (h x 10, -1 = no model) of one pair."""
    kp1, d1, kp2, d2, K, max_iters = job
    q, t, d = oracle.bf_match(d1, d2, 1)
    order = np.argsort(d, kind="stable")
    q, t = q[order], t[order]
    p1 = oracle.keypoints_to_points(kp1[q]).astype(np.float64)
    p2 = oracle.keypoints_to_points(kp2[t]).astype(np.float64)
    m = len(p1)
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    ax, ay = 1. / fx, 1. / fy
    n1 = np.stack([p1[:, 0] * ax + (-cx * ax), p1[:, 1] * ay + (-cy * ay)], 1)
    n2 = np.stack([p2[:, 0] * ax + (-cx * ax), p2[:, 1] * ay + (-cy * ay)], 1)
    thr = 1.0 / ((fx + fy) / 2)
    tf = np.float32(thr * thr)
    cnt = np.full((max_iters, 10), -1, np.int32)
    if m <= 5:
        return m, cnt
    sub = oracle.ransac_subsets(m, max_iters)
    x1, y1, x2, y2 = n1[:, 0], n1[:, 1], n2[:, 0], n2[:, 1]
    for h in range(max_iters):
        Es = oracle.five_point(n1[sub[h]], n2[sub[h]])
        for k, E in enumerate(Es):
            E = E.ravel()
            ex0 = E[0] * x1 + E[1] * y1 + E[2]
            ex1 = E[3] * x1 + E[4] * y1 + E[5]
            ex2 = E[6] * x1 + E[7] * y1 + E[8]
            et0 = E[0] * x2 + E[3] * y2 + E[6]
            et1 = E[1] * x2 + E[4] * y2 + E[7]
            r = x2 * ex0 + y2 * ex1 + ex2
            err = (r * r / (ex0 * ex0 + ex1 * ex1 + et0 * et0 + et1 * et1)).astype(np.float32)
            cnt[h, k] = int(np.sum(err <= tf))
    return m, cnt


def _init():
    os.environ["OMP_NUM_THREADS"] = "1"


def update(ep, niters):
    return oracle.ransac_update_num_iters(0.999, ep, 5, niters)


def replay(m, cnt, max_iters, lo, hi, state):
    """The sequential loop over hypotheses [lo, hi) from state (iter, niters, maxgood)."""
    it, niters, maxgood = state
    h = lo
    while h < hi and it < niters:
        for c in cnt[h]:
            if c < 0:
                break
            if c > max(maxgood, 4):
                maxgood = int(c)
                niters = update((m - c) / m, niters)
        it += 1
        h += 1
    return it, niters, maxgood


def schedule(m, cnt, max_iters, rule):
    """rule(round, h_next, niters, maxgood) -> the round's upper bound (exclusive)."""
    if m <= 5:
        return 0, 0, 0
    state = (0, max_iters, 0)
    h, solved, rounds = 0, 0, 0
    while state[0] < state[1] and h < max_iters:
        hi = min(state[1], rule(rounds, h, state[1], state[2]))
        if hi <= h:
            break
        solved += hi - h
        state = replay(m, cnt, max_iters, h, hi, state)
        h = hi
        rounds += 1
    return state[0], solved, rounds


def main():
    global A
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=256)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--max-iters", type=int, default=1000)
    ap.add_argument("--cache", default="")
    A = ap.parse_args()
    if A.cache and os.path.exists(A.cache):
        z = np.load(A.cache)
        ms, cnts = z["m"], z["cnt"]
    else:
        with Pool(8, initializer=_init) as pool:
            det = pool.map(_detect, range(A.pairs + 1))
            K = det[0][1]
            jobs = [(det[i][0][0], det[i][0][1], det[i + 1][0][0], det[i + 1][0][1], K, A.max_iters)
                    for i in range(A.pairs)]
            res = pool.map(_counts, jobs)
        ms = np.array([r[0] for r in res])
        cnts = np.stack([r[1] for r in res])
        if A.cache:
            np.savez_compressed(A.cache, m=ms, cnt=cnts)
    mi = A.max_iters
    rules = {
        "64 | rest (current)": lambda r, h, n, g: 64 if r == 0 else 1 << 30,
        "64 | 128 | rest": lambda r, h, n, g: [64, 128][r] if r < 2 else 1 << 30,
        "64 | 256 | rest": lambda r, h, n, g: [64, 256][r] if r < 2 else 1 << 30,
        "64 | h+64 | rest": lambda r, h, n, g: 64 if r == 0 else (h + 64 if r == 1 else 1 << 30),
        "64 | h+(n-h)/2 | rest": lambda r, h, n, g: 64 if r == 0 else (h + max(32, (n - h) // 2) if r == 1 else 1 << 30),
        "64 | chunks of 64": lambda r, h, n, g: 64 * (r + 1),
        "64 | chunks of 128": lambda r, h, n, g: 64 + 128 * r,
        "one hypothesis at a time": lambda r, h, n, g: h + 1,
    }
    P = len(ms)
    print(f"{P} pairs, mean matches {ms.mean():.1f}")
    for name, rule in rules.items():
        res = np.array([schedule(ms[p], cnts[p], mi, rule) for p in range(P)])
        it, solved, rounds = res[:, 0], res[:, 1], res[:, 2]
        print(f"{name:28s} iters {it.mean():6.1f}  solved {solved.mean():6.1f} ({solved.mean() / max(it.mean(), 1e-9):.3f}x)"
              f"  rounds max {rounds.max():3d} mean {rounds.mean():5.2f}  pairs in round>=3: {(rounds >= 3).sum()}")
    # niters after round 1 vs final
    res1 = np.array([replay(ms[p], cnts[p], mi, 0, 64, (0, mi, 0)) if ms[p] > 5 else (0, 0, 0) for p in range(P)])
    fin = np.array([schedule(ms[p], cnts[p], mi, rules["one hypothesis at a time"])[0] for p in range(P)])
    need = res1[:, 1] > 64
    print("pairs with niters > 64 after round 1:", int(need.sum()))
    w = np.maximum(0, res1[:, 1] - np.maximum(fin, 64))
    print("waste per pair by niters-after-round-1 bucket:")
    for a, b in ((65, 128), (128, 256), (256, 512), (512, 1001)):
        sel = (res1[:, 1] >= a) & (res1[:, 1] < b)
        print(f"  [{a:4d},{b:4d}): {int(sel.sum()):4d} pairs, waste {w[sel].sum() / P:6.1f} per pair of the batch")


if __name__ == "__main__":
    main()
