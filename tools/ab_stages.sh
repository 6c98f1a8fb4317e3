#!/bin/bash
# One-stream bench of each experiment variant (lib/exp/libdvo_<tag>.so) and the
# product build; per-stage HIP-event times into gpurun_out/ab/<tag>.log.
# usage: tools/ab_stages.sh TAG... [-- bench args]
set -e
tags=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do tags+=("$1"); shift; done; [ "$1" = "--" ] && shift
mkdir -p gpurun_out/ab
for t in base "${tags[@]}"; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --streams 1 --steps 6 --warmup 2 "$@" > gpurun_out/ab/$t.log 2>&1
  echo "$t $(tail -1 gpurun_out/ab/$t.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["stage_ms_per_step"])')"
done
