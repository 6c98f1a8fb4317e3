#!/bin/bash
# Round profile of the default bench command, in two GPU parts (each fits one gpurun call) and a
# merge that runs anywhere:
#   a  rocprofv3 --kernel-trace --stats of the default bench (CPU / drop-in legs off), then
#      separate --pmc passes (FETCH_SIZE; WRITE_SIZE) over a short one-stream bench (batch 512)
#      and over the known-bytes calibration kernels (tools/calib);
#   b  the read-request-size pass (gfx950 TCC_EA0_RDREQ_{32B,64B,128B}: every kernel's fetched
#      bytes, 32 n32 + 64 n64 + 128 n128, whatever its access widths; FETCH_SIZE tallies 128-B
#      requests at 64 B here) over the same short bench and the calibration kernels, then the SQ
#      instruction-count pass;
#   merge  calibration + per-kernel traffic -> gpurun_out/prof/<tag>_pmc_traffic.json.
# usage: tools/profile_round.sh TAG a|b|merge [bench args]
set -e
tag=$1; part=$2; shift 2
root=$(pwd)
out="$root/gpurun_out/prof"
mkdir -p "$out"
# WL: workload flags for every pass (e.g. WL="--width 640 --height 480 --nfeatures 1000"); the merge then
# needs DVO_PMC_CONFIG="640 480 1000" so bench.py finds the document for that workload
short="$WL --steps 1 --warmup 1 --streams 1 --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --no-profile --batch 512"
if [ "$part" = merge ]; then
  python3 "$root/tools/pmc_calibrate.py" "$out/${tag}_calib_known.jsonl" "$out/${tag}_calib_FETCH_SIZE.csv" "$out/${tag}_calib_WRITE_SIZE.csv" "$out/${tag}_pmc_calibration.json" "$out/${tag}_calib_rdreq.csv" > /dev/null
  python3 "$root/tools/pmc_traffic.py" "$out/${tag}_pmc_FETCH_SIZE.csv" "$out/${tag}_pmc_WRITE_SIZE.csv" "$out/${tag}_pmc_sq.csv" "$out/${tag}_pmc_calibration.json" "$out/${tag}_pmc_traffic.json" 512 "$out/${tag}_pmc_rdreq.csv"
  exit 0
fi
export TMPDIR=/tmp
cd /tmp
if [ "$part" = a ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/st_$tag -o run --output-format csv -- python3 "$root/bench.py" --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 "$@" > "$out/${tag}_bench_under_rocprof.log" 2>&1
  python3 "$root/tools/summarize_profile.py" $(find /tmp/st_$tag -name '*kernel_stats.csv') "$out/${tag}_kernel_stats.csv" > "$out/${tag}_kernel_stats.txt"
  for c in FETCH_SIZE WRITE_SIZE; do
    # batch 512: the counter passes serialise every dispatch; traffic per frame is what bench.py scales
    timeout -s KILL 170 rocprofv3 --pmc $c -d /tmp/pmc_${tag}_$c -o run --output-format csv -- python3 "$root/bench.py" $short > "$out/${tag}_pmc_$c.log" 2>&1
    python3 "$root/tools/pmc_summary.py" $(find /tmp/pmc_${tag}_$c -name '*counter_collection.csv') "$out/${tag}_pmc_$c.csv" > /dev/null
    timeout -s KILL 60 rocprofv3 --pmc $c -d /tmp/cal_${tag}_$c -o run --output-format csv -- "$root/tools/calib/build/pmc_calib" > "$out/${tag}_calib_known.jsonl" 2> "$out/${tag}_calib_$c.log"
    python3 "$root/tools/pmc_summary.py" $(find /tmp/cal_${tag}_$c -name '*counter_collection.csv') "$out/${tag}_calib_$c.csv" > /dev/null
  done
elif [ "$part" = b ]; then
  rq="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
  timeout -s KILL 320 rocprofv3 --pmc $rq -d /tmp/pmc_${tag}_rq -o run --output-format csv -- python3 "$root/bench.py" $short > "$out/${tag}_pmc_rdreq.log" 2>&1
  python3 "$root/tools/pmc_summary.py" $(find /tmp/pmc_${tag}_rq -name '*counter_collection.csv') "$out/${tag}_pmc_rdreq.csv" > /dev/null
  timeout -s KILL 60 rocprofv3 --pmc $rq -d /tmp/cal_${tag}_rq -o run --output-format csv -- "$root/tools/calib/build/pmc_calib" > /dev/null 2> "$out/${tag}_calib_rdreq.log"
  python3 "$root/tools/pmc_summary.py" $(find /tmp/cal_${tag}_rq -name '*counter_collection.csv') "$out/${tag}_calib_rdreq.csv" > /dev/null
  timeout -s KILL 170 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d /tmp/pmc_${tag}_sq -o run --output-format csv -- python3 "$root/bench.py" $short > "$out/${tag}_pmc_sq.log" 2>&1
  python3 "$root/tools/pmc_summary.py" $(find /tmp/pmc_${tag}_sq -name '*counter_collection.csv') "$out/${tag}_pmc_sq.csv" > /dev/null
fi
rm -rf /tmp/st_$tag /tmp/pmc_${tag}_* /tmp/cal_${tag}_*
