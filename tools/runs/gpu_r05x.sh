# End-of-round record (continued): two spawned gloo ranks sharing the box's one GPU (batch 1024 per
# rank: two ranks at 3072 exceed one GPU's memory), the sharded path over RCCL at world 1; then the
# Durand-Kerner pass-budget A/B (tools/runs/gpu_r05w.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05v
mkdir -p $O
DVO_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --batch 1024 > $O/bench_gloo_world2_spawned.json 2> $O/bench_gloo.err || exit 1
timeout -k 10 400 python -u bench.py --sharded --cpu-seconds 0 > $O/bench_sharded_rccl_world1.json 2> $O/bench_sharded.err || exit 1
bash tools/runs/gpu_r05w.sh
