# 3.2-mode pyramid through the staged tiles; C2 as main run vs as a config leg
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_opencv32.py tests/test_gpu_edge.py tests/test_gpu_dropin_fused.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
side="--cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0"
timeout -k 10 300 python -u bench.py $side --config-legs c3_ocv32,c2 --runs 3 > $O/bench_legs.json 2> $O/bench_legs.err || exit 1
timeout -k 10 300 python -u bench.py $side --config-legs none --width 640 --height 480 --nfeatures 1000 --runs 3 > $O/bench_c2_main.json 2> $O/bench_c2_main.err || exit 1
