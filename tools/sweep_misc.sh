#!/bin/bash
# A/B of experiment builds (tools/ab_default.sh) plus a few stream/batch
# settings of the product build; one line per configuration in gpurun_out/sw.txt.
# usage: tools/sweep_misc.sh TAG...
set -e
bash tools/ab_default.sh "$@" > gpurun_out/sw_default.txt 2>&1
for cfg in "--streams 3" "--streams 3 --batch 768" "--streams 2 --batch 1536"; do
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --no-profile --steps 12 $cfg > gpurun_out/sw.log 2>&1
  echo "$cfg $(tail -1 gpurun_out/sw.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/sw.txt
done
