# wave priority (s_setprio) of the latency-bound kernels in the two-stream bench: FAST 1 / 3, Durand-Kerner 2,
# FAST 1 + Durand-Kerner 1
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 1000 bash tools/ab_libs.sh fp1 fp3 dk2 fp1dk1 -- --runs 2 > $O/ab.txt 2>&1 || exit 1
