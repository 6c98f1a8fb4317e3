#!/bin/bash
# Round 4: deferred-score parity tests, DK lane-efficiency stats, A/B of the deferred score.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_score_defer.py tests/test_gpu_sampson.py tests/test_gpu_configs.py tests/test_gpu_ransac_parts.py > gpurun_out/r04d_tests.log 2>&1
DVO_LIB_PATH=$PWD/droplet_visual_odometry_amd/lib/exp/libdvo_dkstats.so timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --streams 1 --cpu-seconds 0 --dropin-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --no-profile > gpurun_out/r04d_dkstats.log 2>&1
bash tools/ab_libs.sh nodefer > gpurun_out/r04d_ab.txt 2>&1
