#!/bin/bash
# Round profile of the default bench command: rocprofv3 --kernel-trace --stats,
# then one FETCH_SIZE and one WRITE_SIZE --pmc pass (separate runs, short bench),
# merged into gpurun_out/prof/<tag>_pmc_traffic.json.   usage: tools/profile_round.sh TAG
set -e
tag=$1; shift
root=$(pwd)
out="$root/gpurun_out/prof"
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/st_$tag -o run --output-format csv -- python3 "$root/bench.py" "$@" > "$out/${tag}_bench_under_rocprof.log" 2>&1
python3 "$root/tools/summarize_profile.py" $(find /tmp/st_$tag -name '*kernel_stats.csv') "$out/${tag}_kernel_stats.csv" > "$out/${tag}_kernel_stats.txt"
for c in FETCH_SIZE WRITE_SIZE; do
  # batch 512: the counter passes serialise every dispatch; traffic per frame is what bench.py scales
  timeout -s KILL 170 rocprofv3 --pmc $c -d /tmp/pmc_${tag}_$c -o run --output-format csv -- python3 "$root/bench.py" --steps 1 --warmup 1 --streams 1 --cpu-seconds 0 --no-profile --batch 512 > "$out/${tag}_pmc_$c.log" 2>&1
  python3 "$root/tools/pmc_summary.py" $(find /tmp/pmc_${tag}_$c -name '*counter_collection.csv') "$out/${tag}_pmc_$c.csv" > /dev/null
done
python3 "$root/tools/pmc_traffic.py" "$out/${tag}_pmc_FETCH_SIZE.csv" "$out/${tag}_pmc_WRITE_SIZE.csv" "$out/${tag}_pmc_traffic.json" 512
rm -rf /tmp/st_$tag /tmp/pmc_${tag}_*
