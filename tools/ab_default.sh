#!/bin/bash
# Default two-stream bench of the product build and each experiment variant
# (lib/exp/libdvo_<tag>.so via DVO_LIB_PATH): whole-pipeline frames/s.
# usage: tools/ab_default.sh TAG... [-- bench args]
set -e
tags=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do tags+=("$1"); shift; done; [ "$1" = "--" ] && shift
mkdir -p gpurun_out/ab
for t in base "${tags[@]}" base; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --no-profile --steps 16 "$@" > gpurun_out/ab/d_$t.log 2>&1
  echo "$t $(tail -1 gpurun_out/ab/d_$t.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
