#!/bin/bash
# Kernel trace of a short one-stream bench; per-(kernel, grid) means into gpurun_out/trace/<tag>.txt
set -e
tag=$1; shift
root=$(pwd)
mkdir -p "$root/gpurun_out/trace"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tr_$tag -o run --output-format csv -- python3 "$root/bench.py" --steps 3 --warmup 1 --streams 1 --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --no-profile "$@" > "$root/gpurun_out/trace/${tag}.log" 2>&1
python3 "$root/tools/trace_summary.py" $(find /tmp/tr_$tag -name '*kernel_trace.csv') "$root/gpurun_out/trace/${tag}.txt" > /dev/null
rm -rf /tmp/tr_$tag
