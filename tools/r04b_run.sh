set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pairs.py tests/test_gpu_pose_tail.py tests/test_gpu_opencv32.py > gpurun_out/r04b_tests.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err
