set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pipeline.py > gpurun_out/r05d_gpu_pipeline.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r05d_gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > gpurun_out/r05d_bench.json 2> gpurun_out/r05d_bench.err
