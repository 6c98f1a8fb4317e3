# Durand-Kerner lane refill (DVO_DK_REFILL): parity of rf, then A/B at C3 and C2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06g
mkdir -p $O
DVO_LIB_PATH=$PWD/droplet_visual_odometry_amd/lib/exp/libdvo_rf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_ransac_parts.py tests/test_gpu_score_defer.py tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_rf.log 2>&1 || exit 1
DVO_LIB_PATH=$PWD/droplet_visual_odometry_amd/lib/exp/libdvo_rf2p.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_rf2p.log 2>&1 || exit 1
timeout -k 10 900 bash tools/ab_libs.sh rf rf32 rfp2 rf2p -- --runs 2 > $O/ab_c3.txt 2>&1 || exit 1
timeout -k 10 600 bash tools/ab_libs.sh rf rf2p -- --runs 2 --width 640 --height 480 --nfeatures 1000 > $O/ab_c2.txt 2>&1 || exit 1
