"""Regenerate the committed golden fixtures (run from the repo root):

    python tests/golden/make_golden.py

pair_320x240.npz   two seeded synthetic 320x240 frames and the oracle's outputs
                   for the whole per-pair path (ORB keypoints/descriptors,
                   sorted cross-checked matches, E, R, t, cheirality count,
                   RANSAC iterations).  Frames are stored, not re-rendered.
notes_kat1.json    KAT-1: the 10 logged matches (20 keypoint coordinates) from
                   /root/reference/scripts/back_up_files/frame_extraction_notes.txt:6-7,
                   real OpenCV ORB output on 1400x1080 frames, transcribed as numbers.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# frame_extraction_notes.txt:6-7 — (prev kp, cur kp, distance) of the 10 top matches
NOTES_KAT1 = [
    ((722.6083374023438, 382.2060546875), (892.8094482421875, 412.06591796875), 2.0),
    ((914.4000244140625, 660.9600219726562), (727.2000122070312, 452.1600036621094), 3.0),
    ((731.5662841796875, 447.897705078125), (752.4681396484375, 653.9306640625), 3.0),
    ((901.7673950195312, 641.9867553710938), (695.7344360351562, 391.16400146484375), 3.0),
    ((718.800048828125, 567.6000366210938), (698.4000244140625, 632.4000244140625), 4.0),
    ((758.9378051757812, 579.7786865234375), (935.6085205078125, 472.7809143066406), 4.0),
    ((737.5382690429688, 621.0848388671875), (722.6083374023438, 367.276123046875), 4.0),
    ((931.6272583007812, 465.8136291503906), (695.1372680664062, 394.1499938964844), 4.0),
    ((728.4000244140625, 378.0), (757.2000122070312, 655.2000122070312), 5.0),
    ((860.9589233398438, 427.99114990234375), (694.241455078125, 629.5451049804688), 5.0),
]


def main():
    import oracle
    from droplet_visual_odometry_amd.synth import SceneStream
    oracle.build()
    st = SceneStream(320, 240)
    frames = np.stack([st.render(i).numpy() for i in (0, 1)])
    K = st.K
    kp0, d0 = oracle.detect_and_compute(frames[0], 300)
    r = oracle.pair_pose(frames[0], frames[1], K, 300, kp_prev=(kp0, d0))
    np.savez_compressed(os.path.join(HERE, "pair_320x240.npz"), frames=frames, K=K, nfeatures=300,
                        kp0=kp0, desc0=d0, kp1=r["kp_cur"], desc1=r["desc_cur"], q=r["q"], t=r["t"],
                        p1=r["p1"], p2=r["p2"], E=r["E"], R=r["R"], t_unit=r["t_unit"], good=r["good"],
                        iters=r["iters"])
    with open(os.path.join(HERE, "notes_kat1.json"), "w") as f:
        json.dump({"source": "scripts/back_up_files/frame_extraction_notes.txt:6-7",
                   "matches": [{"prev": list(a), "cur": list(b), "distance": d} for a, b, d in NOTES_KAT1]}, f,
                  indent=1)
    print("golden written:", len(kp0), len(r["kp_cur"]), "kps,", len(r["q"]), "matches, iters", r["iters"])


if __name__ == "__main__":
    main()
