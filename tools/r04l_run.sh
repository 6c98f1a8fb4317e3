#!/bin/bash
# Round 4: FAST writes the descriptor blur of its tiles (DVO_FAST_BLUR); describe reads it.
set -e
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/debug/fast_blur_diff.py 1280 720 > gpurun_out/r04l_diff.txt 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fast_blur.py tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_opencv32.py tests/test_gpu_dropin_fused.py > gpurun_out/r04l_tests.log 2>&1
bash tools/ab_default.sh nofb fbw5 fbfirst pkb > gpurun_out/r04l_ab.txt 2>&1
