# Durand-Kerner lane refill: every later pass vs the last pass only, persistent grids of 768 / 384 blocks; C3 and C2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 900 bash tools/ab_libs.sh rf rfl rf384 rfl384 -- --runs 2 > $O/ab_c3.txt 2>&1 || exit 1
timeout -k 10 700 bash tools/ab_libs.sh rf rfl rf384 rfl384 -- --runs 2 --width 640 --height 480 --nfeatures 1000 > $O/ab_c2.txt 2>&1 || exit 1
