#!/bin/bash
# Round 4: queue Durand-Kerner -- parity tests, lane stats, A/B against the pass kernel and IPL / ring variants.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_ransac_parts.py tests/test_gpu_score_defer.py tests/test_gpu_pairs.py tests/test_gpu_sharded.py > gpurun_out/r04e_tests.log 2>&1
DVO_LIB_PATH=$PWD/droplet_visual_odometry_amd/lib/exp/libdvo_dkqstats.so timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --streams 1 --cpu-seconds 0 --dropin-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --no-profile > gpurun_out/r04e_dkstats.log 2>&1
bash tools/ab_libs.sh passes noring ipl4 ipl12 ipl16 > gpurun_out/r04e_ab.txt 2>&1
