set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sharded.py tests/test_gpu_pipeline.py > gpurun_out/r05f_gpu_sharded.log 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05f_bench_default.json 2> gpurun_out/r05f_bench_default.err &&
DVO_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --batch 1024 --cpu-seconds 4 > gpurun_out/r05f_bench_gloo2.json 2> gpurun_out/r05f_bench_gloo2.err &&
timeout -k 10 300 python -u bench.py --sharded --steps 10 --warmup 2 --cpu-seconds 2 --pose-check-per-rank 3 > gpurun_out/r05f_bench_rccl1.json 2> gpurun_out/r05f_bench_rccl1.err
