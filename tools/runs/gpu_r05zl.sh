# The r05zk matcher variant (ci) vs the product build (base) at C2 (640x480, 1000 features) and C5
# (1920x1080, 4000 features, 4096 iterations, B 1024), side legs off, alternating twice
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zl
mkdir -p $O
side="--cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 --runs 3"
for t in base ci base ci; do
  for c in c2 c5; do
    lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
    if [ $c = c2 ]; then wl="--width 640 --height 480 --nfeatures 1000"; else wl="--width 1920 --height 1080 --nfeatures 4000 --max-iters 4096 --batch 1024"; fi
    DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py $wl $side > $O/${c}_$t.json 2> $O/${c}_$t.err || exit 1
    python3 -c "
import json
d=json.loads([l for l in open('$O/${c}_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('$c $t', d['value'], d['ms_per_step'], d['runs']['frames_per_s'], 'match', round(st.get('match'), 3))" >> $O/ab.txt
  done
done
