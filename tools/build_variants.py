"""Build experiment variants of libdvo_hip.so (lib/exp/libdvo_<tag>.so) from
`-D` macro sets, for A/B stage timing on the GPU box via DVO_LIB_PATH.
usage: python tools/build_variants.py TAG=MACRO[,MACRO...] ...
(a spec containing '|' is split on '|' instead, for macro values with commas:
 r3='DVO_RANSAC_BOUNDS=64,256,1073741824|' -- the '|' is required for those)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from droplet_visual_odometry_amd.build import LIBDIR, build  # noqa: E402

for spec in sys.argv[1:]:
    tag, _, macros = spec.partition("=")
    out = os.path.join(LIBDIR, "exp", f"libdvo_{tag}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    sep = "|" if "|" in macros else ","
    print(build(force=True, out=out, defines=[m for m in macros.split(sep) if m]))
