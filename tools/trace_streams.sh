#!/bin/bash
# Kernel trace of the default (multi-stream) bench; concurrency summary into gpurun_out/trace/<tag>_timeline.txt
set -e
tag=$1; shift
root=$(pwd)
mkdir -p "$root/gpurun_out/trace"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tl_$tag -o run --output-format csv -- python3 "$root/bench.py" --steps 4 --warmup 1 --cpu-seconds 0 --no-profile "$@" > "$root/gpurun_out/trace/${tag}_tl.log" 2>&1
python3 "$root/tools/trace_timeline.py" $(find /tmp/tl_$tag -name '*kernel_trace.csv') "$root/gpurun_out/trace/${tag}_timeline.txt" > /dev/null
rm -rf /tmp/tl_$tag
