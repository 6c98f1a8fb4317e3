"""Build the duplicate-launch experiment variants for tools/ab_dup.sh.

usage: python tools/ab_dup.py build MASK...   (masks: dvo_internal.h kDup*)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from droplet_visual_odometry_amd import build as B  # noqa: E402


def main(argv):
    assert argv and argv[0] == "build", __doc__
    os.makedirs(os.path.join(B.LIBDIR, "exp"), exist_ok=True)
    for m in argv[1:]:
        out = os.path.join(B.LIBDIR, "exp", f"libdvo_dup{m}.so")
        print(B.build(out=out, defines=[f"DVO_EXP_DUP={m}"]))


if __name__ == "__main__":
    main(sys.argv[1:])
