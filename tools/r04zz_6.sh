#!/bin/bash
# Round 4: pairs-vs-stream equality at 300 pairs (frame groups in both schedules), then the default bench line.
set -e
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pairs.py > gpurun_out/prof/r04zz_pairs_tests.log 2>&1
timeout -k 10 600 python3 -u bench.py > gpurun_out/prof/r04zz_bench_default.json 2> gpurun_out/prof/r04zz_bench_default.err
