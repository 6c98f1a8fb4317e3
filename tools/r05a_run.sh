#!/bin/bash
# End of round 4, candidates for round 5 (not adopted): FAST waves per EU 5 / 7, Harris frame groups
# 1 / 4, ORB detection groups 192 / 384, against the product build at C3 (B 3072) and C2.
set -e
mkdir -p gpurun_out
bash tools/ab_default.sh fw5 fw7 hg1 hg4 g192 g384 > gpurun_out/r05a_ab.txt 2>&1
bash tools/ab_default.sh fw5 fw7 g192 g384 -- --width 640 --height 480 --nfeatures 1000 > gpurun_out/r05a_ab_c2.txt 2>&1
