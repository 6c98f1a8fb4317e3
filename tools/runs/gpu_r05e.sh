set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_default.sh b48 b6 b4 b64 -- --runs 3 > gpurun_out/r05e_ab_c3_bounds.txt 2>&1 &&
bash tools/ab_default.sh b48 b6 b4 b64 -- --runs 3 --width 640 --height 480 --nfeatures 1000 > gpurun_out/r05e_ab_c2_bounds.txt 2>&1
