# sharded tests (gather to rank 0, reset_pose), the default bench as the driver runs it, eight gloo
# ranks on the box's one GPU, the sharded path over RCCL at world 1
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
DVO_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 8 --batch 256 > $O/bench_gloo_world8_b256.json 2> $O/bench_gloo8.err || exit 1
timeout -k 10 300 python -u bench.py --sharded --cpu-seconds 0 > $O/bench_sharded_rccl_world1.json 2> $O/bench_sharded.err || exit 1
