"""Per-call timing of the detector entry points (host image in, keypoints and
descriptors out, as the drop-in calls them) on the GPU, beside the oracle's
single-thread time for the same frame.  usage: python tools/time_detectors.py"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def timeit(fn, reps):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return 1e3 * (time.perf_counter() - t) / reps


def main():
    from conftest import synth_frames
    import oracle
    from droplet_visual_odometry_amd import ops
    oracle.use_native_build()
    out = []
    for W, H in ((640, 480), (1280, 720)):
        img = synth_frames(W, H, range(1))[0][0]
        row = {"size": f"{W}x{H}"}
        for name, gpu, cpu in (
                ("orb_2000", lambda: ops.detect_and_compute(img, 2000), lambda: oracle.detect_and_compute(img, 2000)),
                ("sift", lambda: ops.sift_detect_and_compute(img), lambda: oracle.sift_detect_and_compute(img)),
                ("surf_400", lambda: ops.surf_detect_and_compute(img, 400.0),
                 lambda: oracle.surf_detect_and_compute(img, 400.0))):
            n = len(gpu()[0])
            row[name] = {"keypoints": n, "gpu_ms": round(timeit(gpu, 20), 3), "oracle_1t_ms": round(timeit(cpu, 2), 1)}
        out.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
