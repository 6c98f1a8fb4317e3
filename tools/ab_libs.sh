#!/bin/bash
# Default (two-stream) bench of the product build and of experiment variants
# lib/exp/libdvo_<tag>.so, alternating, two rounds.  usage: tools/ab_libs.sh TAG... [-- bench args]
set -e
tags=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do tags+=("$1"); shift; done; [ "$1" = "--" ] && shift
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for t in base "${tags[@]}"; do
    lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
    DVO_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --steps 10 --warmup 2 "$@" > gpurun_out/ab/${t}_$rep.log 2>&1
    echo "$t rep $rep $(tail -1 gpurun_out/ab/${t}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"] or {}; print(d["value"], d["ms_per_step"], {k: round(v, 2) for k, v in r.get("stage_ms_per_step", {}).items()})')"
  done
done
