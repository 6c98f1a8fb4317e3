#!/bin/bash
# Round 4: level-0 select at 256 threads (new default): GPU tests; then the batch / streams sweep of the product build.
set -e
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_opencv32.py tests/test_gpu_dropin.py tests/test_gpu_dropin_fused.py tests/test_gpu_pairs.py > gpurun_out/r04u_tests.log 2>&1
for args in "--batch 2048" "--batch 3072" "--batch 4096" "--streams 3" "--batch 2048"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 300 python -u bench.py --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --no-profile --steps 16 --dropin-seconds 0 $args > gpurun_out/ab/u_$tag.log 2>&1
  echo "$args $(tail -1 gpurun_out/ab/u_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/r04u_sweep.txt
done
