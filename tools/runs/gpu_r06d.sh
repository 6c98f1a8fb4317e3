# FAST one wave per strip (DVO_FAST_WAVE=1, lib/exp/libdvo_fw.so): parity on the detection tests, then
# the default two-stream bench alternating with the product build
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06d
mkdir -p $O
DVO_LIB_PATH=$PWD/droplet_visual_odometry_amd/lib/exp/libdvo_fw.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_opencv32.py tests/test_gpu_configs.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_fw.log 2>&1 || exit 1
timeout -k 10 900 bash tools/ab_libs.sh fw -- --runs 3 > $O/ab.txt 2>&1 || exit 1
