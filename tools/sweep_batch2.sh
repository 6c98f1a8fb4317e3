#!/bin/bash
# Two-stream bench at several batch sizes / stream counts (10 steps, no CPU legs).
# usage: tools/sweep_batch2.sh "B:S ..."  -> gpurun_out/sweep/<B>_<S>.json
set -e
mkdir -p gpurun_out/sweep
for bs in $1; do
  b=${bs%%:*}; s=${bs##*:}
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --steps 10 --warmup 2 --batch $b --streams $s > gpurun_out/sweep/${b}_${s}.json 2> gpurun_out/sweep/${b}_${s}.err
  echo "$b $s $(python3 -c "import json; d=json.load(open('gpurun_out/sweep/${b}_${s}.json')); print(d['value'], d['ms_per_step'])")"
done
