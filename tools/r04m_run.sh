#!/bin/bash
# Round 4: recoverPose [R|t] / [R|-t] from one triangulation (DVO_POSE_MIRROR); matcher packed backward keys (pkb variant).
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r04m_tests.log 2>&1
bash tools/ab_default.sh nomirror pkb > gpurun_out/r04m_ab.txt 2>&1
bash tools/ab_stages.sh nomirror pkb -- --dropin-seconds 0 > gpurun_out/r04m_ab_one_stream.txt 2>&1
