#!/bin/bash
# Kernel trace of the bench on ONE stream; the last batch's kernel sequence into
# gpurun_out/trace/<tag>_sequence.txt.   usage: tools/trace_one_stream.sh TAG [bench args]
set -e
tag=$1; shift
root=$(pwd)
mkdir -p "$root/gpurun_out/trace"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/seq_$tag -o run --output-format csv -- python3 "$root/bench.py" --steps 3 --warmup 1 --streams 1 --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --no-profile "$@" > "$root/gpurun_out/trace/${tag}_seq.log" 2>&1
python3 "$root/tools/trace_sequence.py" $(find /tmp/seq_$tag -name '*kernel_trace.csv') "$root/gpurun_out/trace/${tag}_sequence.txt" > /dev/null
rm -rf /tmp/seq_$tag
