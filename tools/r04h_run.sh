#!/bin/bash
# Round 4: score early-exit A/B (pyramid back on the single-level kernel), then the fused drop-in /
# sharded / rank-0 tail checks (r04f).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pyramid.py tests/test_gpu_dropin_fused.py > gpurun_out/r04h_tests.log 2>&1
bash tools/ab_libs.sh nobail > gpurun_out/r04h_ab.txt 2>&1
bash tools/r04f_run.sh
