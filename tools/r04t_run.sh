#!/bin/bash
# Round 4: select_fast level-0 block width, repeat: s256 / s192 against the 128-thread base, two passes.
set -e
mkdir -p gpurun_out
bash tools/ab_default.sh s256 s192 > gpurun_out/r04t_ab.txt 2>&1
bash tools/ab_default.sh s256 s192 > gpurun_out/r04t_ab2.txt 2>&1
bash tools/ab_stages.sh s256 -- --dropin-seconds 0 > gpurun_out/r04t_ab_one_stream.txt 2>&1
