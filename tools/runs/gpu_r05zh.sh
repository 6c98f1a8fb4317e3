# FAST as a persistent grid of 4 (p4) or 5 (p5) workgroups per CU, leaving the rest of each CU to the
# other stream, vs the product build (base); ORB parity tests on p4 first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05zh
mkdir -p $O
for t in; do
  DVO_LIB_PATH=$PWD/droplet_visual_odometry_amd/lib/exp/libdvo_$t.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_opencv32.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_$t.log 2>&1 || exit 1
done
for t in base p4 p5 base p4 p5; do
  lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > $O/d_$t.json 2> $O/d_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('$O/d_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('$t', d['value'], d['ms_per_step'], d['runs']['frames_per_s'], 'fast', st.get('fast'), 'describe', st.get('describe'))" >> $O/ab.txt
done
