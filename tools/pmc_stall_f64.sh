#!/bin/bash
# Two SQ counter passes over a short one-stream bench (batch 512): the stall
# breakdown (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES) and the
# f64 VALU instruction counts (FMA / MUL / ADD / TRANS) that bench.py's
# RANSAC f64-issue fraction is priced from.  Summaries into
# gpurun_out/prof/<tag>_pmc_{stall,f64}.csv.   usage: tools/pmc_stall_f64.sh TAG [bench args]
set -e
tag=$1; shift
root=$(pwd)
out="$root/gpurun_out/prof"
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
short="$WL --steps 1 --warmup 1 --streams 1 --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --no-profile --batch 512"
timeout -s KILL 170 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
  -d /tmp/pmc_${tag}_stall -o run --output-format csv -- python3 "$root/bench.py" $short "$@" > "$out/${tag}_pmc_stall.log" 2>&1
python3 "$root/tools/pmc_summary.py" $(find /tmp/pmc_${tag}_stall -name '*counter_collection.csv') "$out/${tag}_pmc_stall.csv" > /dev/null
timeout -s KILL 170 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES \
  -d /tmp/pmc_${tag}_f64 -o run --output-format csv -- python3 "$root/bench.py" $short "$@" > "$out/${tag}_pmc_f64.log" 2>&1
python3 "$root/tools/pmc_summary.py" $(find /tmp/pmc_${tag}_f64 -name '*counter_collection.csv') "$out/${tag}_pmc_f64.csv" > /dev/null
# Durand-Kerner per pass: the f64 pass's per-dispatch counts against a counter-free kernel trace of the same bench
timeout -k 10 170 rocprofv3 --kernel-trace -d /tmp/pmc_${tag}_kt -o run --output-format csv -- python3 "$root/bench.py" $short "$@" > "$out/${tag}_dk_trace.log" 2>&1
python3 "$root/tools/dk_passes.py" $(find /tmp/pmc_${tag}_f64 -name '*counter_collection.csv') $(find /tmp/pmc_${tag}_kt -name '*kernel_trace.csv') "$out/${tag}_dk_passes.json" > "$out/${tag}_dk_passes.txt"
rm -rf /tmp/pmc_${tag}_*
