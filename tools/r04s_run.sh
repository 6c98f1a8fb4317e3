#!/bin/bash
# Round 4: RANSAC round bounds re-measured on the current tree (base 64/inf, r3a 64/256/inf, r3b 64/160/inf,
# r2c 48/inf) at C3 and C2; select_fast's level-0 blocks at 256 / 512 / 1024 threads (sN).
set -e
mkdir -p gpurun_out
bash tools/ab_default.sh r3a r3b r2c s256 s512 s1024 > gpurun_out/r04s_ab.txt 2>&1
bash tools/ab_default.sh r3a r3b r2c -- --width 640 --height 480 --nfeatures 1000 > gpurun_out/r04s_ab_c2.txt 2>&1
