# FAST occupancy: the compass word list inside each wave's candidate segment (LDS 26.0 -> 23.0 KB) at
# 6 (o6) and 7 (o7) waves per SIMD, vs the product build (base); ORB parity tests on o7 first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05z
mkdir -p $O
for t in o7 o6; do
  DVO_LIB_PATH=$PWD/droplet_visual_odometry_amd/lib/exp/libdvo_$t.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_opencv32.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_$t.log 2>&1 || exit 1
done
for t in base o6 o7 base o6 o7; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > $O/d_$t.json 2> $O/d_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('$O/d_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('$t', d['value'], d['ms_per_step'], d['runs']['frames_per_s'], 'fast', st.get('fast'), 'describe', st.get('describe'))" >> $O/ab.txt
done
for t in base o7; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --streams 1 --steps 8 --warmup 4 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > $O/s1_$t.json 2> $O/s1_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('$O/s1_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('one-stream $t', d['value'], d['ms_per_step'], 'fast', st.get('fast'), 'describe', st.get('describe'))" >> $O/ab.txt
done
