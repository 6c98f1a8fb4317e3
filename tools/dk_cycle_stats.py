"""Durand-Kerner sweep statistics of the RANSAC polynomials of the bench
stream (solvePoly, mathfuncs.cpp: 300 Gauss-Seidel sweeps unless maxDiff
reaches 0).  For each five-point polynomial of the first hypotheses of each
pair the oracle's per-sweep root-state hashes give: the natural exit (maxDiff
== 0), the pre-period mu and period lambda of the limit cycle the roots fall
into, and the sweeps each exit rule runs:
  brent     the device's DkBrent (snapshots at powers of two, then on to the
            sweep congruent to 300 mod lambda)
  ideal     a detector that sees the first repeated state (mu + lambda), then
            runs on to the congruent sweep
  oracle    what solvePoly itself runs (300, or the natural exit)

usage: python tools/dk_cycle_stats.py [--pairs 24] [--hyps 64] [--width 1280 --height 720 --nfeatures 2000]"""
import argparse
import ctypes
import os
import sys
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

A = None


def _init():
    import torch
    torch.set_num_threads(1)


def _detect(i):
    from droplet_visual_odometry_amd.synth import SceneStream
    st = SceneStream(A.width, A.height)
    return oracle.detect_and_compute(st.render(i).numpy(), A.nfeatures), st.K


def brent_sweeps(tr, nat):
    """DkBrent on the hash sequence: state after sweep k is tr[k-1] (state 0 = start, hashed as None)."""
    saved, saved_it, power, target = None, 0, 1, 300
    it = 0
    while True:
        it += 1
        if it >= nat:  # natural exit (maxDiff == 0) at sweep nat
            return it
        if it >= target:
            return it
        cur = tr[it - 1]
        if target == 300:
            if saved is not None and cur == saved:
                target = it + (300 - it) % (it - saved_it)
                if it >= target:
                    return it
            elif it - saved_it == power:
                saved, saved_it = cur, it
                power <<= 1


def _poly_stats(job):
    kp1, d1, kp2, d2, K, hyps = job
    L = oracle.lib()
    L.ora_last_five_point_poly.argtypes = [ctypes.c_void_p]
    L.ora_solve_poly_trace.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    q, t, d = oracle.bf_match(d1, d2, 1)
    order = np.argsort(d, kind="stable")
    q, t = q[order], t[order]
    p1 = oracle.keypoints_to_points(kp1[q]).astype(np.float64)
    p2 = oracle.keypoints_to_points(kp2[t]).astype(np.float64)
    m = len(p1)
    if m <= 5:
        return []
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    ax, ay = 1. / fx, 1. / fy
    n1 = np.stack([p1[:, 0] * ax + (-cx * ax), p1[:, 1] * ay + (-cy * ay)], 1)
    n2 = np.stack([p2[:, 0] * ax + (-cx * ax), p2[:, 1] * ay + (-cy * ay)], 1)
    sub = oracle.ransac_subsets(m, hyps)
    out = []
    c = np.zeros(11)
    tr = np.zeros(301, np.uint64)
    for h in range(hyps):
        oracle.five_point(n1[sub[h]], n2[sub[h]])
        L.ora_last_five_point_poly(c.ctypes.data)
        n = L.ora_solve_poly_trace(c.ctypes.data, 10, 300, tr.ctypes.data)
        if n != 10:
            continue
        nat = int(tr[300])
        seq = [int(x) for x in tr[:nat]]
        first = {}
        mu = lam = -1
        for k, hv in enumerate(seq):
            if hv in first:
                mu, lam = first[hv] + 1, k - first[hv]  # state after sweep mu+lam == after sweep mu
                break
            first[hv] = k
        b = brent_sweeps(seq, nat if nat < 300 else 10 ** 9)
        if mu >= 0:
            k = mu + lam
            ideal = k + (300 - k) % lam
        else:
            ideal = nat
        out.append((nat, mu, lam, b, min(ideal, nat)))
    return out


def main():
    global A
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=24)
    ap.add_argument("--hyps", type=int, default=64)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--dump", default="", help="save (natural, mu, lambda, brent, ideal) per polynomial (.npy)")
    A = ap.parse_args()
    with Pool(8, initializer=_init) as pool:
        det = pool.map(_detect, range(A.pairs + 1))
        K = det[0][1]
        jobs = [(det[i][0][0], det[i][0][1], det[i + 1][0][0], det[i + 1][0][1], K, A.hyps) for i in range(A.pairs)]
        res = [r for part in pool.map(_poly_stats, jobs) for r in part]
    a = np.array(res)
    if A.dump:
        np.save(A.dump, a)
    nat, mu, lam, brent, ideal = a.T
    cyc = mu >= 0
    print(f"{len(a)} polynomials ({A.pairs} pairs x {A.hyps} hypotheses, {A.width}x{A.height}, N={A.nfeatures})")
    print(f"natural exit (maxDiff == 0) before 300: {np.mean(nat < 300):.3f}; cycling: {np.mean(cyc):.3f}; "
          f"neither (300 sweeps, no repeat): {np.mean((nat >= 300) & ~cyc):.3f}")
    print(f"mean sweeps: oracle {nat.mean():.1f}  brent {brent.mean():.1f}  ideal {ideal.mean():.1f}")
    for name, v in (("mu", mu[cyc]), ("lambda", lam[cyc]), ("brent", brent), ("ideal", ideal), ("natural", nat)):
        print(f"  {name:8s} percentiles 10/25/50/75/90/99: {np.percentile(v, [10, 25, 50, 75, 90, 99])}")
    print("lambda histogram (cycling):", np.bincount(np.minimum(lam[cyc], 40).astype(int))[1:].tolist())
    for thr in (48, 128):
        print(f"  fraction still running after {thr}: brent {np.mean(brent > thr):.3f}  ideal {np.mean(ideal > thr):.3f}")


if __name__ == "__main__":
    main()
