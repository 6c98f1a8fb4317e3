"""Where one fused drop-in pair's time goes (D7): content hashes of both frames,
the library call (ops.PairStream.pair: upload, detect, match, RANSAC,
recoverPose, record back), and the host tail (_relative_transform:
triangulatePoints + numpy), over a synthetic 1280x720 / 2000-feature stream.
usage: python tools/profile_fused.py [seconds]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "droplet_visual_odometry_amd", "dropin"))
import visual_odometry_v3 as v3  # noqa: E402
from droplet_visual_odometry_amd.synth import MARKER_LEN, SceneStream  # noqa: E402


def main(seconds=4.0):
    sc = SceneStream(1280, 720, device="cuda")
    frames = [sc.render(i).cpu().numpy() for i in range(48)]
    cs = [sc.marker_corners(i) for i in range(48)]
    import tempfile
    d = ", ".join(repr(float(v)) for v in np.asarray(sc.K).ravel())
    with tempfile.NamedTemporaryFile("w", suffix=".yaml", delete=False) as fh:
        fh.write(f"camera_matrix:\n  rows: 3\n  cols: 3\n  data: [{d}]\n"
                 "distortion_coefficients:\n  rows: 1\n  cols: 5\n  data: [0.0, 0.0, 0.0, 0.0, 0.0]\n")
    vo = v3.VisualOdometry(mode="orb", calibration_file_path=fh.name, controlled=True, real_marker_length=MARKER_LEN)
    os.unlink(fh.name)
    vo.feature_detector.setMaxFeatures(2000)
    T = vo.robot_curr_position
    vo.visual_odometry_calculations(frames[0], frames[1], T, cs[0], cs[1])
    ps = vo._pair_engine[1]
    t_hash, t_call, t_tail, n = [], [], [], 0
    last = None
    t_end = time.perf_counter() + seconds
    i = 1
    while time.perf_counter() < t_end:
        a = i % 47
        t0 = time.perf_counter()
        kp, kc = v3._FeatureCache.key(frames[a]), v3._FeatureCache.key(frames[a + 1])
        t1 = time.perf_counter()
        rec = ps.pair(None if last == kp else frames[a], frames[a + 1], reuse_prev=last == kp)
        last = kc
        t2 = time.perf_counter()
        vo._relative_transform(rec["R"].reshape(3, 3).copy(), rec["t"].reshape(3, 1).copy(), cs[a], cs[a + 1])
        t3 = time.perf_counter()
        t_hash.append(t1 - t0)
        t_call.append(t2 - t1)
        t_tail.append(t3 - t2)
        i += 1
    med = lambda x: 1e3 * float(np.median(x))  # noqa: E731
    print(f"pairs {len(t_call)}: hash {med(t_hash):.3f} ms, library call {med(t_call):.3f} ms, "
          f"host tail {med(t_tail):.3f} ms (medians)")


if __name__ == "__main__":
    main(float(sys.argv[1]) if len(sys.argv) > 1 else 4.0)
