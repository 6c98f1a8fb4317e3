#!/bin/bash
# Round 4: FAST with three barriers per tile (DVO_FAST_3BAR, base) vs four (bar4); detection groups on in both.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_opencv32.py tests/test_gpu_dropin.py tests/test_gpu_dropin_fused.py tests/test_gpu_pairs.py > gpurun_out/r04r_tests.log 2>&1
bash tools/ab_default.sh bar4 > gpurun_out/r04r_ab.txt 2>&1
bash tools/ab_default.sh bar4 > gpurun_out/r04r_ab2.txt 2>&1
bash tools/ab_stages.sh bar4 -- --dropin-seconds 0 > gpurun_out/r04r_ab_one_stream.txt 2>&1
