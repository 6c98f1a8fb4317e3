set -o pipefail
cd $GRAFT_REPO_ROOT
for q in 4 8 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python -u bench.py --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --dropin-seconds 0 --pose-check-32 0 --tail-world 0 > gpurun_out/r05h_q$q.json 2> gpurun_out/r05h_q$q.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r05h_q$q.json') if l.startswith('{')][-1])
print('queues $q', d['value'], d['legs']['host_fed'].get('value'), d['legs']['host_fed'].get('ms_per_step'))" >> gpurun_out/r05h_queues.txt
done
