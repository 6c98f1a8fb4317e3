#!/bin/bash
# Round 4: describe phase 2 fast sincos (fdlibm kernels, float-rounding-safe, ocml fallback) and DPP wave sums.
# head = previous commit's build; nosc = this tree without the fast sincos; gN = detection over groups of N frames (DVO_ORB_GROUP).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_configs.py tests/test_gpu_opencv32.py tests/test_gpu_dropin.py tests/test_gpu_dropin_fused.py > gpurun_out/r04o_tests.log 2>&1
bash tools/ab_default.sh head nosc g64 g128 g256 > gpurun_out/r04o_ab.txt 2>&1
bash tools/ab_stages.sh head nosc g128 -- --dropin-seconds 0 > gpurun_out/r04o_ab_one_stream.txt 2>&1
