#!/bin/bash
# SQ counter passes over a short bench run (one stream, no CPU leg); summaries
# into gpurun_out/pmc/<tag>_sq{1,2}.csv.   usage: tools/pmc_sq.sh TAG [bench args]
set -e
tag=$1; shift
root=$(pwd)
mkdir -p "$root/gpurun_out/pmc"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  -d /tmp/pmc_$tag.1 -o run --output-format csv -- python3 "$root/bench.py" --steps 2 --warmup 1 --streams 1 --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --no-profile "$@" > "$root/gpurun_out/pmc/${tag}_b1.log" 2>&1
python3 "$root/tools/pmc_summary.py" $(find /tmp/pmc_$tag.1 -name '*counter_collection.csv') "$root/gpurun_out/pmc/${tag}_sq1.csv"
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE \
  -d /tmp/pmc_$tag.2 -o run --output-format csv -- python3 "$root/bench.py" --steps 2 --warmup 1 --streams 1 --cpu-seconds 0 --config-legs none --no-ref-equivalent --no-host-fed --tail-world 0 --no-profile "$@" > "$root/gpurun_out/pmc/${tag}_b2.log" 2>&1
python3 "$root/tools/pmc_summary.py" $(find /tmp/pmc_$tag.2 -name '*counter_collection.csv') "$root/gpurun_out/pmc/${tag}_sq2.csv"
