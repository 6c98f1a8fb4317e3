# FAST workgroups per CU capped by reserved dynamic LDS: 6 (base), 5 (l5: +6.5 KB), 4 (l4: +14.5 KB), leaving LDS
# for the other stream's kernels on the same CUs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zd
mkdir -p $O
for t in base l5 l4 base l5 l4; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > $O/d_$t.json 2> $O/d_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('$O/d_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('$t', d['value'], d['ms_per_step'], d['runs']['frames_per_s'], 'fast', st.get('fast'), 'describe', st.get('describe'), 'ransac', st.get('ransac'))" >> $O/ab.txt
done
