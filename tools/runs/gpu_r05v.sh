# End-of-round record on the final tree: GPU suite, smoke, default bench (every leg), C2, C5, two
# spawned gloo ranks on the box's one GPU, the sharded path over RCCL at world 1
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 400 python -u bench.py --width 640 --height 480 --nfeatures 1000 > $O/bench_640x480_n1000.json 2> $O/bench_640x480_n1000.err || exit 1
timeout -k 10 500 python -u bench.py --width 1920 --height 1080 --nfeatures 4000 --max-iters 4096 --batch 1024 > $O/bench_1920x1080_n4000_it4096_b1024.json 2> $O/bench_c5.err || exit 1
DVO_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 > $O/bench_gloo_world2_spawned.json 2> $O/bench_gloo.err || exit 1
timeout -k 10 400 python -u bench.py --sharded --cpu-seconds 0 > $O/bench_sharded_rccl_world1.json 2> $O/bench_sharded.err || exit 1
