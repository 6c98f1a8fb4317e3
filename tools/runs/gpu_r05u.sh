# stage C over a real-root mask + Durand-Kerner records by item + matcher two-half key fold = base; HEAD = c0; base without the matcher change = m0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05u
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05u/gpu_tests.log 2>&1 || exit 1
for t in base c0 m0 base c0 m0; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > gpurun_out/r05u/d_$t.json 2> gpurun_out/r05u/d_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r05u/d_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('$t', d['value'], d['ms_per_step'], d['runs']['frames_per_s'], 'ransac', st.get('ransac'), 'match', st.get('match'))" >> gpurun_out/r05u/ab.txt
done
