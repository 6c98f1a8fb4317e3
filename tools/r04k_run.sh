#!/bin/bash
# Round 4 checkpoint: full GPU suite, then the kernel-stats + default bench record of this tree.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r04k_tests.log 2>&1
bash tools/stats_and_bench.sh r04k
