# Matcher stages of 32 trains (ci32: a barrier per 32 trains, 8 KB of LDS per workgroup) on top of the
# r05zk C-input keys (ci), vs ci and the product build (base); the whole GPU suite on ci32 first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zn
mkdir -p $O
DVO_LIB_PATH=$PWD/droplet_visual_odometry_amd/lib/exp/libdvo_ci32.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_ci32.log 2>&1 || exit 1
for t in base ci ci32 base ci ci32; do
  lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > $O/d_$t.json 2> $O/d_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('$O/d_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('$t', d['value'], d['ms_per_step'], d['runs']['frames_per_s'], 'match', st.get('match'), 'fast', st.get('fast'), 'describe', st.get('describe'))" >> $O/ab.txt
done
