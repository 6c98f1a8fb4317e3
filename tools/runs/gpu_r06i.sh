# matcher trains prefetched two stages ahead (pf2), describe two keypoints per wave (dkw2): parity of pf2,
# A/B at C3 and C5
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06i
mkdir -p $O
DVO_LIB_PATH=$PWD/droplet_visual_odometry_amd/lib/exp/libdvo_pf2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin_fused.py tests/test_gpu_pipeline.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_pf2.log 2>&1 || exit 1
DVO_LIB_PATH=$PWD/droplet_visual_odometry_amd/lib/exp/libdvo_dkw2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_dkw2.log 2>&1 || exit 1
timeout -k 10 700 bash tools/ab_libs.sh pf2 dkw2 -- --runs 2 > $O/ab_c3.txt 2>&1 || exit 1
timeout -k 10 500 bash tools/ab_libs.sh pf2 -- --runs 2 --width 1920 --height 1080 --nfeatures 4000 --max-iters 4096 --batch 1024 > $O/ab_c5.txt 2>&1 || exit 1
