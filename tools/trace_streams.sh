#!/bin/bash
# Kernel trace of the default (two-stream) bench and the overlap report of its
# last batches into gpurun_out/trace/<tag>_overlap.txt.  usage: tools/trace_streams.sh TAG [bench args]
set -e
tag=$1; shift
root=$(pwd)
mkdir -p "$root/gpurun_out/trace"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/ovl_$tag -o run --output-format csv -- python3 "$root/bench.py" --steps 6 --warmup 2 --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --no-profile "$@" > "$root/gpurun_out/trace/${tag}_ovl.log" 2>&1
python3 "$root/tools/trace_overlap.py" $(find /tmp/ovl_$tag -name '*kernel_trace.csv') "$root/gpurun_out/trace/${tag}_overlap.txt" > /dev/null
python3 -c "
import csv, gzip, sys
src = sys.argv[1]
with open(src) as f, gzip.open(sys.argv[2], 'wt') as g:
    r = csv.DictReader(f)
    w = csv.DictWriter(g, fieldnames=['Kernel_Name', 'Start_Timestamp', 'End_Timestamp'], extrasaction='ignore')
    w.writeheader()
    for row in r:
        if 'dvo::' in row.get('Kernel_Name', ''):
            w.writerow(row)
" $(find /tmp/ovl_$tag -name '*kernel_trace.csv') "$root/gpurun_out/trace/${tag}_dvo_kernels.csv.gz"
rm -rf /tmp/ovl_$tag
