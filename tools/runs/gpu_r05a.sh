set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dropin_fused.py tests/test_gpu_sharded.py tests/test_gpu_dropin.py > gpurun_out/r05a_gpu_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05a_bench_default.json 2> gpurun_out/r05a_bench_default.err &&
(timeout -k 10 60 python -u bench.py --gpus 2 --steps 2 > gpurun_out/r05a_nccl2_refused.log 2>&1; echo "rc=$?" >> gpurun_out/r05a_nccl2_refused.log; true) &&
DVO_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --batch 1024 --cpu-seconds 4 > gpurun_out/r05a_bench_gloo2.json 2> gpurun_out/r05a_bench_gloo2.err
