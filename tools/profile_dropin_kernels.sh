#!/bin/bash
# Kernel stats of the drop-in per-pair surface (tools/profile_dropin.py under
# rocprofv3 --kernel-trace --stats) into gpurun_out/prof/<tag>_dropin_kernels.txt.
# usage: tools/profile_dropin_kernels.sh TAG
set -e
tag=$1
root=$(pwd)
out="$root/gpurun_out/prof"
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/dk_$tag -o run --output-format csv -- python3 "$root/tools/profile_dropin.py" > "$out/${tag}_dropin_profile.log" 2>&1
python3 "$root/tools/summarize_profile.py" $(find /tmp/dk_$tag -name '*kernel_stats.csv') "$out/${tag}_dropin_kernel_stats.csv" > "$out/${tag}_dropin_kernels.txt"
rm -rf /tmp/dk_$tag
