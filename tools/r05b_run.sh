#!/bin/bash
# End of round 4: ORB detection group size 384 / 512 / 768 / none (g0) against the product's 256,
# at C3 (B 3072) and C2, after r05a showed 384 ahead of 256.
set -e
mkdir -p gpurun_out
bash tools/ab_default.sh g384 g512 g768 g0 g384 > gpurun_out/r05b_ab.txt 2>&1
bash tools/ab_default.sh g384 g512 g768 g0 g384 -- --width 640 --height 480 --nfeatures 1000 > gpurun_out/r05b_ab_c2.txt 2>&1
