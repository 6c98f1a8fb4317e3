#!/bin/bash
# Round 4 final tree: stall + f64 passes (+ Durand-Kerner per pass) at C3, C2 (640x480/1000) and C5 (1920x1080/4000, 4096 hypotheses).
set -e
bash tools/pmc_stall_f64.sh r04zz
WL="--width 640 --height 480 --nfeatures 1000" bash tools/pmc_stall_f64.sh r04zzc2
WL="--width 1920 --height 1080 --nfeatures 4000 --max-iters 4096" bash tools/pmc_stall_f64.sh r04zzc5
