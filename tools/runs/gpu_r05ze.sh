# select_harris on an LDS copy of each level's list for batches (cap 2048 / 1024) vs the global-memory path (base)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ze
mkdir -p $O
DVO_LIB_PATH=$PWD/droplet_visual_odometry_amd/lib/exp/libdvo_h2k.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_opencv32.py tests/test_gpu_pipeline.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_h2k.log 2>&1 || exit 1
for t in base h2k h1k base h2k h1k; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > $O/d_$t.json 2> $O/d_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('$O/d_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('$t', d['value'], d['ms_per_step'], d['runs']['frames_per_s'], 'select_harris', st.get('select_harris'), 'fast', st.get('fast'))" >> $O/ab.txt
done
