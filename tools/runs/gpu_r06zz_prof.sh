# Round 6 profile of the final tree at the bench's configuration: usage DVO_TREE=<commit> bash tools/runs/gpu_r06zz_prof.sh a|b1|b2|c|d
#   a / b1 / b2: tools/profile_final.sh parts at C3 (B 3072); c: kernel stats of the C2 and C5 configurations;
#   d: kernel stats of a bench whose only config leg is c3_ocv32 (its <true> kernels are the 3.2 leg's)
set -o pipefail
cd $GRAFT_REPO_ROOT
case "$1" in
  a|b1|b2) timeout -k 10 1150 bash tools/profile_final.sh r06zz "$1" || exit 1 ;;
  c)
    export TMPDIR=/tmp
    out=$GRAFT_REPO_ROOT/gpurun_out/prof
    mkdir -p $out
    side="--cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 --config-legs none"
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/st_c2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --width 640 --height 480 --nfeatures 1000 $side > $out/r06zzc2_bench_under_rocprof.log 2>&1) || exit 1
    python3 tools/summarize_profile.py $(find /tmp/st_c2 -name '*kernel_stats.csv') $out/r06zzc2_kernel_stats.csv > $out/r06zzc2_kernel_stats.txt || exit 1
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/st_c5 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --width 1920 --height 1080 --nfeatures 4000 --max-iters 4096 --batch 1024 $side > $out/r06zzc5_bench_under_rocprof.log 2>&1) || exit 1
    python3 tools/summarize_profile.py $(find /tmp/st_c5 -name '*kernel_stats.csv') $out/r06zzc5_kernel_stats.csv > $out/r06zzc5_kernel_stats.txt || exit 1
    rm -rf /tmp/st_c2 /tmp/st_c5 ;;
  d)
    export TMPDIR=/tmp
    out=$GRAFT_REPO_ROOT/gpurun_out/prof
    mkdir -p $out
    side="--cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --leg-runs 1"
    (cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/st_c3o -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --config-legs c3_ocv32 $side > $out/r06zzc3o_bench_under_rocprof.log 2>&1) || exit 1
    python3 tools/summarize_profile.py $(find /tmp/st_c3o -name '*kernel_stats.csv') $out/r06zzc3o_kernel_stats.csv > $out/r06zzc3o_kernel_stats.txt || exit 1
    rm -rf /tmp/st_c3o ;;
esac
