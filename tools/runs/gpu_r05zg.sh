# RANSAC score hypotheses per block: 16 (base) vs 8 / 32 (DVO_SCORE_HYPS)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zg
mkdir -p $O
for t in base sh8 sh32 base sh8 sh32; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > $O/d_$t.json 2> $O/d_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('$O/d_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('$t', d['value'], d['ms_per_step'], d['runs']['frames_per_s'], 'fast', st.get('fast'), 'describe', st.get('describe'), 'ransac', st.get('ransac'))" >> $O/ab.txt
done
