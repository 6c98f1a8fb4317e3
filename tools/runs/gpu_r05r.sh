# pyramid in sub-launches of 128 / 256 frames (level l+1 reads level l from the MALL) vs whole group;
# then: does a rocprofv3 --pmc pass over the bench complete with 4 HW queues?
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05r
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05r/gpu_tests.log 2>&1 || exit 1
for t in base h0 p128 p256 base h0 p128 p256; do
  lib=droplet_visual_odometry_amd/lib/libdvo_hip.so; [ "$t" != base ] && lib=droplet_visual_odometry_amd/lib/exp/libdvo_$t.so
  DVO_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 > gpurun_out/r05r/d_$t.json 2> gpurun_out/r05r/d_$t.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r05r/d_$t.json') if l.startswith('{')][-1])
st=d['roofline']['stage_ms_per_step']
print('$t', d['value'], d['ms_per_step'], d['runs']['frames_per_s'], 'pyramid', st.get('pyramid'), 'ransac', st.get('ransac'))" >> gpurun_out/r05r/ab.txt
done
cd /tmp
export TMPDIR=/tmp
side="--cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 --steps 1 --warmup 1 --runs 1 --no-profile --streams 1"
( time GPU_MAX_HW_QUEUES=4 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d /tmp/q4 -o run --output-format csv -- python3 $R/bench.py $side --batch 512 ) > $R/gpurun_out/r05r/q4_b512.log 2>&1 || exit 1
ls -la $(find /tmp/q4 -name '*counter_collection.csv') > $R/gpurun_out/r05r/files.txt
