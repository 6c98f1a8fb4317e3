# FAST: score, NMS and output of a tile on one rotating wave (3 barriers per tile) = base, vs HEAD (f0)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05y
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05y/gpu_tests.log 2>&1 || exit 1
for t in base f0 base f0; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > gpurun_out/r05y/d_$t.json 2> gpurun_out/r05y/d_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r05y/d_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('$t', d['value'], d['ms_per_step'], d['runs']['frames_per_s'], 'fast', st.get('fast'), 'match', st.get('match'))" >> gpurun_out/r05y/ab.txt
done
for t in base f0; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --streams 1 --steps 8 --warmup 4 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > gpurun_out/r05y/s1_$t.json 2> gpurun_out/r05y/s1_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r05y/s1_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('one-stream $t', d['value'], d['ms_per_step'], 'stages', st)" >> gpurun_out/r05y/ab.txt
done
