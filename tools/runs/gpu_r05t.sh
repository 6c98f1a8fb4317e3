# RANSAC stage A / C over packed items (dk_off) instead of 64-hypothesis blocks per pair (base) vs
# HEAD (a0); GPU suite first; then one default bench with every leg (rank-0 tail leg with per-buffer waits)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05t
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05t/gpu_tests.log 2>&1 || exit 1
for t in base a0 base a0; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > gpurun_out/r05t/d_$t.json 2> gpurun_out/r05t/d_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r05t/d_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('$t', d['value'], d['ms_per_step'], d['runs']['frames_per_s'], 'ransac', st.get('ransac'), 'fast', st.get('fast'))" >> gpurun_out/r05t/ab.txt
done
timeout -k 10 400 python -u bench.py > gpurun_out/r05t/bench_default.json 2> gpurun_out/r05t/bench_default.err || exit 1
