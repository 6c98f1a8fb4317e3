# RANSAC score: two points per lane with packed f32 (decide2, paired point layout) = base, vs HEAD (s0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05zb
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05zb/gpu_tests.log 2>&1 || exit 1
for t in base s0 base s0; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > gpurun_out/r05zb/d_$t.json 2> gpurun_out/r05zb/d_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r05zb/d_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('$t', d['value'], d['ms_per_step'], d['runs']['frames_per_s'], 'ransac', st.get('ransac'), 'fast', st.get('fast'))" >> gpurun_out/r05zb/ab.txt
done
for t in base s0; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --streams 1 --steps 8 --warmup 4 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > gpurun_out/r05zb/s1_$t.json 2> gpurun_out/r05zb/s1_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r05zb/s1_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('one-stream $t', d['value'], d['ms_per_step'], 'ransac', st.get('ransac'))" >> gpurun_out/r05zb/ab.txt
done
