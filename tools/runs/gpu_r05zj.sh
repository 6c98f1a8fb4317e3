# Knob re-sweep on the round-5 kernels: Harris keypoint groups per wave (hg1/3/4; product 2) and RANSAC
# score points per LDS chunk (sc128/512; product 256), two-stream default bench, alternating twice
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zj
mkdir -p $O
for t in base hg1 hg3 hg4 sc128 sc512 base hg1 hg3 hg4 sc128 sc512; do
  lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > $O/d_$t.json 2> $O/d_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('$O/d_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('$t', d['value'], d['ms_per_step'], d['runs']['frames_per_s'], {k: round(v, 3) for k, v in st.items()})" >> $O/ab.txt
done
