#!/bin/bash
# Kernel-trace profile of the float k-NN matcher (tools/bench_knn.py) into
# gpurun_out/prof/<tag>_knn_*; copy the summaries to profiles/.
set -e
tag=${1:-knn}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/knn_$tag -o run --output-format csv -- python3 tools/bench_knn.py > gpurun_out/prof/${tag}_knn_bench.log 2>&1
cp "$(find /tmp/knn_$tag -name '*kernel_stats.csv')" gpurun_out/prof/${tag}_knn_kernel_stats.csv
