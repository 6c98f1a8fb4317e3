# Round 6 record on the final tree: GPU suite, smoke, the default bench as the driver runs it (every leg,
# config legs included), eight gloo ranks on the box's one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06zz
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
DVO_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 8 --batch 256 > $O/bench_gloo_world8_b256.json 2> $O/bench_gloo8.err || exit 1
