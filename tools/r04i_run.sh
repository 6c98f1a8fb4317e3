#!/bin/bash
# Round 4: quad-DPP pose chain -- tests, rank-0 tail rehearsal; fused drop-in time breakdown.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pose_tail.py tests/test_gpu_sharded.py tests/test_gpu_pairs.py > gpurun_out/r04i_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --dropin-seconds 0 > gpurun_out/r04i_tail.json 2> gpurun_out/r04i_tail.err
timeout -k 10 200 python -u tools/profile_fused.py 4 > gpurun_out/r04i_fused_profile.txt 2>&1
