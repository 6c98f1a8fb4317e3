#!/bin/bash
# rank 0's world-8 tail leg (bench.py legs.rank0_tail_world8) for the product build and variants
# usage: tools/ab_tail.sh TAG... [-- bench args]
set -e
tags=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do tags+=("$1"); shift; done; [ "$1" = "--" ] && shift
mkdir -p gpurun_out/ab
for t in base "${tags[@]}" base; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --cpu-seconds 0 --no-ref-equivalent --no-host-fed --dropin-seconds 0 --pose-check-32 0 --config-legs none --no-profile --runs 1 --steps 16 "$@" > gpurun_out/ab/t_$t.log 2>&1
  echo "$t $(tail -1 gpurun_out/ab/t_$t.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); l=d["legs"]["rank0_tail_world8"]; print(d["value"], l["ms_per_step_without_tail"], l["ms_per_step_with_tail"], l["added_frac"], l["tail_alone_ms"])')"
done
