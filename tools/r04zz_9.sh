#!/bin/bash
# Round 4: the sharded bench path on the final tree: RCCL at world 1 (--sharded, default batch) and two gloo ranks
# sharing the box's one GPU (batch 1024), as the driver's N > 1 runs take it.
set -e
mkdir -p gpurun_out/prof
timeout -k 10 400 python3 -u bench.py --sharded --steps 6 --warmup 2 --cpu-seconds 0 --dropin-seconds 0 > gpurun_out/prof/r04zz_bench_sharded_rccl_world1.json 2> gpurun_out/prof/r04zz_bench_sharded_rccl_world1.err
DVO_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --batch 1024 --steps 4 --warmup 1 --cpu-seconds 0 --dropin-seconds 0 > gpurun_out/prof/r04zz_bench_gloo_world2.json 2> gpurun_out/prof/r04zz_bench_gloo_world2.err
