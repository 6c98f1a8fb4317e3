set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sharded.py tests/test_gpu_pose_tail.py > gpurun_out/r05l_gpu_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 12 --warmup 5 --runs 1 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --dropin-seconds 0 --pose-check-32 0 > gpurun_out/r05l_tail.json 2> gpurun_out/r05l_tail.err
