#!/bin/bash
# Throughput of the default pipeline over batch sizes / streams (no profiling, no CPU leg).
set -e
mkdir -p gpurun_out/sweep
for cfg in "--batch 512" "--batch 768" "--batch 1024" "--batch 1024 --streams 3" "--batch 512 --streams 3"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --no-profile --steps 16 $cfg > gpurun_out/sweep/$tag.log 2>&1
  echo "$cfg $(tail -1 gpurun_out/sweep/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
