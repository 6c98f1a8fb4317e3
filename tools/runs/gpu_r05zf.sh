# kernel stats of the C2 and C5 bench configurations on the final tree (rocprofv3 --kernel-trace --stats)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
side="--cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/st_c2 -o run --output-format csv -- python3 $R/bench.py --width 640 --height 480 --nfeatures 1000 $side > $O/r05zzc2_bench_under_rocprof.log 2>&1 || exit 1
python3 $R/tools/summarize_profile.py $(find /tmp/st_c2 -name '*kernel_stats.csv') $O/r05zzc2_kernel_stats.csv > $O/r05zzc2_kernel_stats.txt || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/st_c5 -o run --output-format csv -- python3 $R/bench.py --width 1920 --height 1080 --nfeatures 4000 --max-iters 4096 --batch 1024 $side > $O/r05zzc5_bench_under_rocprof.log 2>&1 || exit 1
python3 $R/tools/summarize_profile.py $(find /tmp/st_c5 -name '*kernel_stats.csv') $O/r05zzc5_kernel_stats.csv > $O/r05zzc5_kernel_stats.txt || exit 1
rm -rf /tmp/st_c2 /tmp/st_c5
