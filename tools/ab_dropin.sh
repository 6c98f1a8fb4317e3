#!/bin/bash
# Drop-in per-pair rate (tools/profile_dropin.py's first, un-profiled leg) of the product
# build and of experiment variants lib/exp/libdvo_<tag>.so.  usage: tools/ab_dropin.sh TAG...
set -e
mkdir -p gpurun_out/ab
for t in base "$@"; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 120 python -u tools/profile_dropin.py > gpurun_out/ab/dropin_$t.log 2>&1
  echo "$t $(grep -m1 dropin_pairs_per_s gpurun_out/ab/dropin_$t.log)"
done
