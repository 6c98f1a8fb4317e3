#!/bin/bash
# Round 4: pose chain (prefetched chunks, unrolled), fused pair call (one-launch feature rotation, pinned uploads).
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pose_tail.py tests/test_gpu_sharded.py tests/test_gpu_dropin_fused.py tests/test_gpu_dropin.py > gpurun_out/r04j_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --dropin-seconds 5 > gpurun_out/r04j_bench.json 2> gpurun_out/r04j_bench.err
timeout -k 10 200 python -u tools/profile_fused.py 4 > gpurun_out/r04j_fused_profile.txt 2>&1
