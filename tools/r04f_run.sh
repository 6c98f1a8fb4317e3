#!/bin/bash
# Round 4: fused drop-in pair path -- tests and the drop-in rate.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dropin_fused.py tests/test_gpu_dropin.py tests/test_gpu_parity.py tests/test_gpu_edge.py > gpurun_out/r04f_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 5 > gpurun_out/r04f_bench.json 2> gpurun_out/r04f_bench.err
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sharded.py > gpurun_out/r04f_sharded.log 2>&1
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --dropin-seconds 0 > gpurun_out/r04f_tail.json 2> gpurun_out/r04f_tail.err
