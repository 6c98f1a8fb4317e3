set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "3072 2" "4096 2" "3072 3" "2048 3" "2048 2" "3072 2"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --batch $1 --streams $2 --steps 12 --warmup 5 --runs 3 --cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 --no-profile > gpurun_out/r05m_b$1_s$2.json 2> gpurun_out/r05m_b$1_s$2.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r05m_b$1_s$2.json') if l.startswith('{')][-1])
print('batch $1 streams $2', d['value'], d['ms_per_step'], d['runs']['frames_per_s'])" >> gpurun_out/r05m_sweep.txt
done
