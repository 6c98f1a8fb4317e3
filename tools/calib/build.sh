#!/bin/bash
# Builds the PMC calibration binary (run on the GPU box under rocprofv3 --pmc).
set -e
here=$(cd "$(dirname "$0")" && pwd)
mkdir -p "$here/build"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -x hip -o "$here/build/pmc_calib" "$here/pmc_calib.cpp"
