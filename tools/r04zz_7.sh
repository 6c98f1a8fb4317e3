#!/bin/bash
# Round 4 final default bench line (reference-equivalent check ordered after its frame gather).
set -e
mkdir -p gpurun_out/prof
timeout -k 10 600 python3 -u bench.py > gpurun_out/prof/r04zz_bench_default.json 2> gpurun_out/prof/r04zz_bench_default.err
