#!/bin/bash
# Round 4: detection over frame groups (DVO_ORB_GROUP = 256 / 512 / 1024) against the whole batch (base), two passes.
set -e
mkdir -p gpurun_out
bash tools/ab_default.sh g256 g512 g1024 > gpurun_out/r04p_ab.txt 2>&1
bash tools/ab_default.sh g256 g512 g1024 > gpurun_out/r04p_ab2.txt 2>&1
