# Durand-Kerner pass budgets on the pipelined rounds: base 48 / 80 / rest; k1 48 / 48 / 96 / rest;
# k2 40 / 60 / rest; k3 64 / 96 / rest (DVO_DK_B0..B2)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05w
for t in base k1 k2 k3 base k1 k2 k3; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > gpurun_out/r05w/d_$t.json 2> gpurun_out/r05w/d_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r05w/d_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('$t', d['value'], d['ms_per_step'], d['runs']['frames_per_s'], 'ransac', st.get('ransac'))" >> gpurun_out/r05w/ab.txt
done
