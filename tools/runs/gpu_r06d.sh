# FAST one wave per strip (DVO_FAST_WAVE=1, lib/exp/libdvo_fw.so) against the product build: the default
# two-stream bench alternating (parity of the variant: r06d/gpu_tests_fw.log, 80 passed)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 900 bash tools/ab_libs.sh fw -- --runs 3 > $O/ab.txt 2>&1 || exit 1
