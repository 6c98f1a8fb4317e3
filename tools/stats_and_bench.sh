#!/bin/bash
# End-of-session record: rocprofv3 --kernel-trace --stats of the default bench command
# (CPU and drop-in legs off) and the default bench itself, into gpurun_out/prof/<tag>_*.
# usage: tools/stats_and_bench.sh TAG
set -e
tag=$1
root=$(pwd)
out="$root/gpurun_out/prof"
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/st_$tag -o run --output-format csv -- python3 "$root/bench.py" --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 > "$out/${tag}_bench_under_rocprof.log" 2>&1
python3 "$root/tools/summarize_profile.py" $(find /tmp/st_$tag -name '*kernel_stats.csv') "$out/${tag}_kernel_stats.csv" > "$out/${tag}_kernel_stats.txt"
rm -rf /tmp/st_$tag
cd "$root"
timeout -k 10 400 python3 -u bench.py > "$out/${tag}_bench_default.json" 2> "$out/${tag}_bench_default.err"
