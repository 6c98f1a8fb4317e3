#!/bin/bash
# Default-bench frames/s over (streams, batch) shapes (no CPU / drop-in legs, no stage events).
# usage: tools/sweep_streams.sh "CFG1" "CFG2" ...   (each CFG a string of bench.py flags)
set -e
mkdir -p gpurun_out/sweep
for cfg in "$@"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --no-profile --steps 8 $cfg > gpurun_out/sweep/$tag.log 2>&1
  echo "$cfg $(tail -1 gpurun_out/sweep/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
