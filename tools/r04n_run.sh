#!/bin/bash
# Round 4: describe ICAngles: disk masks from a constant table (icloop), moments by v_dot4 on LDS words (base); head = the previous commit's build.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_opencv32.py tests/test_gpu_dropin.py tests/test_gpu_dropin_fused.py > gpurun_out/r04n_tests.log 2>&1
bash tools/ab_default.sh head icloop > gpurun_out/r04n_ab.txt 2>&1
bash tools/ab_stages.sh head icloop -- --dropin-seconds 0 > gpurun_out/r04n_ab_one_stream.txt 2>&1
