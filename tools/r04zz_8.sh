#!/bin/bash
# Round 4: final source tree (RANSAC experiment switches pruned; generated code identical): full GPU suite + smoke.
set -e
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/prof/r04zz_gpu_tests_final.log 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/prof/r04zz_smoke_final.log 2>&1
