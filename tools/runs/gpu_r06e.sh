# FAST wave variants: 16-row sub-tiles, describe at wave priority 2 (alone and with the wave FAST);
# parity of fw16p, two-stream A/B, then one-stream stage times
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06e
mkdir -p $O
DVO_LIB_PATH=$PWD/droplet_visual_odometry_amd/lib/exp/libdvo_fw16p.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_opencv32.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_fw16p.log 2>&1 || exit 1
timeout -k 10 900 bash tools/ab_libs.sh fwp fw16p bp -- --runs 2 > $O/ab.txt 2>&1 || exit 1
timeout -k 10 600 bash tools/ab_libs.sh fw fw16p -- --runs 2 --streams 1 --batch 2048 > $O/ab_one_stream.txt 2>&1 || exit 1
