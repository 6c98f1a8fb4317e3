"""Writes data/sift_exp_tab.inc: the 64-entry table of cv::hal::exp32f's scalar
path (mathfuncs_core: expTab[i] = 2^(i/64) * EXPPOLY_32F_A0, used as float),
shared by the SIFT oracle (oracle/sift.cpp) and the device kernels
(csrc/sift.hip) so both evaluate exp() with the same float operations."""
import os

A0 = .9670371139572337719125840413672004409288e-2
rows = [float.hex(2.0 ** (i / 64.0) * A0) for i in range(64)]
out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "sift_exp_tab.inc")
with open(out, "w") as f:
    f.write("// expTab of cv::hal::exp32f: 2^(i/64) * EXPPOLY_32F_A0 as doubles (tools/gen_exp_table.py)\n")
    for i in range(0, 64, 4):
        f.write("    " + ", ".join(rows[i:i + 4]) + ",\n")
