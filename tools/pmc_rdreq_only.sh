#!/bin/bash
# The request-size PMC pass alone (see profile_round.sh): TCC_EA0_RDREQ_{32B,64B,128B} over the
# calibration kernels and a short bench, into gpurun_out/prof/<tag>_{calib,pmc}_rdreq.csv.
# usage: tools/pmc_rdreq_only.sh TAG
set -e
tag=$1
root=$(pwd)
out="$root/gpurun_out/prof"
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
rq="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
timeout -s KILL 60 rocprofv3 --pmc $rq -d /tmp/cal_${tag}_rq -o run --output-format csv -- "$root/tools/calib/build/pmc_calib" > "$out/${tag}_calib_known.jsonl" 2> "$out/${tag}_calib_rdreq.log"
python3 "$root/tools/pmc_summary.py" $(find /tmp/cal_${tag}_rq -name '*counter_collection.csv') "$out/${tag}_calib_rdreq.csv"
short="--steps 1 --warmup 1 --streams 1 --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --no-profile --batch 512"
timeout -s KILL 320 rocprofv3 --pmc $rq -d /tmp/pmc_${tag}_rq -o run --output-format csv -- python3 "$root/bench.py" $short > "$out/${tag}_pmc_rdreq.log" 2>&1
python3 "$root/tools/pmc_summary.py" $(find /tmp/pmc_${tag}_rq -name '*counter_collection.csv') "$out/${tag}_pmc_rdreq.csv" > /dev/null
rm -rf /tmp/pmc_${tag}_* /tmp/cal_${tag}_*
