#!/bin/bash
# Marginal cost of kernels in the default two-stream bench: each variant
# lib/exp/libdvo_dup<mask>.so launches the kernels of DVO_EXP_DUP=<mask> twice
# (idempotent ones; dvo_internal.h), so value(base) - value(variant) is what one
# more copy of them costs with the other stream overlapping.  Build the variants
# on the CPU first: python tools/ab_dup.py build MASK...
# usage: tools/ab_dup.sh MASK... ; results in gpurun_out/ab/dup_<mask>.log
set -e
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for m in 0 "$@"; do
    lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$m" != 0 ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_dup$m.so
    DVO_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --cpu-seconds 0 --dropin-seconds 0 --no-profile --steps 10 --warmup 2 > gpurun_out/ab/dup_${m}_$rep.log 2>&1
    echo "dup $m rep $rep $(tail -1 gpurun_out/ab/dup_${m}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
