#!/bin/bash
# Round 4 final tree: traffic / SQ passes at C2 and C5 (for their bench lines' roofline.traffic).
set -e
WL="--width 640 --height 480 --nfeatures 1000" bash tools/profile_round.sh r04zzc2 a --width 640 --height 480 --nfeatures 1000
WL="--width 640 --height 480 --nfeatures 1000" bash tools/profile_round.sh r04zzc2 b
WL="--width 1920 --height 1080 --nfeatures 4000 --max-iters 4096" bash tools/profile_round.sh r04zzc5 a --width 1920 --height 1080 --nfeatures 4000 --max-iters 4096 --batch 1024
WL="--width 1920 --height 1080 --nfeatures 4000 --max-iters 4096" bash tools/profile_round.sh r04zzc5 b
