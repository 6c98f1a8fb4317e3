#!/bin/bash
# Round 4 after adopting ORB detection groups of 768: GPU suite, smoke, default / C2 / C5 bench lines.
set -e
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/prof/r04zzz_gpu_tests.log 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/prof/r04zzz_smoke.log 2>&1
timeout -k 10 600 python3 -u bench.py > gpurun_out/prof/r04zzz_bench_default.json 2> gpurun_out/prof/r04zzz_bench_default.err
timeout -k 10 400 python3 -u bench.py --width 640 --height 480 --nfeatures 1000 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 > gpurun_out/prof/r04zzz_bench_640x480_n1000.json 2> gpurun_out/prof/r04zzz_bench_640x480_n1000.err
timeout -k 10 500 python3 -u bench.py --width 1920 --height 1080 --nfeatures 4000 --max-iters 4096 --batch 1024 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 > gpurun_out/prof/r04zzz_bench_1920x1080_n4000_it4096_b1024.json 2> gpurun_out/prof/r04zzz_bench_1920x1080_n4000_it4096_b1024.err
