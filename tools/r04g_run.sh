#!/bin/bash
# Round 4: two-level pyramid parity + A/B, then the fused drop-in / sharded / tail checks (r04f).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pyramid.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_score_defer.py tests/test_gpu_ransac_parts.py > gpurun_out/r04g_tests.log 2>&1
bash tools/ab_libs.sh onelevel nobail > gpurun_out/r04g_ab.txt 2>&1
bash tools/r04f_run.sh
