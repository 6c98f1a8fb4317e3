#!/bin/bash
# rocprofv3 kernel trace of one bench.py run: the dvo:: dispatches (name, grid, queue / stream,
# start, end) into gpurun_out/trace/<tag>_trace.csv.gz and the per-(kernel, grid) means into
# gpurun_out/trace/<tag>_summary.txt.   usage: tools/trace_run.sh TAG [bench args]
set -e
tag=$1; shift
root=$(pwd)
mkdir -p "$root/gpurun_out/trace"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/tr_$tag -o run --output-format csv -- python3 "$root/bench.py" --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 --config-legs none --no-profile --runs 1 "$@" > "$root/gpurun_out/trace/${tag}.log" 2>&1
csv=$(find /tmp/tr_$tag -name '*kernel_trace.csv')
python3 "$root/tools/trace_summary.py" $csv "$root/gpurun_out/trace/${tag}_summary.txt" > /dev/null
python3 - $csv "$root/gpurun_out/trace/${tag}_trace.csv.gz" <<'PY'
import csv, gzip, sys
with open(sys.argv[1]) as f, gzip.open(sys.argv[2], 'wt') as g:
    r = csv.DictReader(f)
    keep = [k for k in r.fieldnames if k in ('Kernel_Name', 'Start_Timestamp', 'End_Timestamp', 'Queue_Id', 'Stream_Id',
                                                 'Grid_Size_X', 'Grid_Size_Y', 'Grid_Size_Z', 'Grid_Size', 'Correlation_Id')]
    w = csv.DictWriter(g, fieldnames=keep, extrasaction='ignore')
    w.writeheader()
    for row in r:
        if 'dvo::' in row.get('Kernel_Name', ''):
            w.writerow(row)
PY
rm -rf /tmp/tr_$tag
