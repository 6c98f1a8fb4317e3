#!/bin/bash
# Round 4: detection in balanced frame groups of <= 256 (DVO_ORB_GROUP default) with per-group stage
# events; full GPU suite, A/B against the whole-batch build (g0), one-stream stage times.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r04q_gpu_tests.log 2>&1
bash tools/ab_default.sh g0 > gpurun_out/r04q_ab.txt 2>&1
bash tools/ab_stages.sh g0 -- --dropin-seconds 0 > gpurun_out/r04q_ab_one_stream.txt 2>&1
