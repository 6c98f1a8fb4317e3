set -e
mkdir -p gpurun_out/sweep
for cfg in "--streams 1" "--streams 2" "--streams 3" "--streams 4" "--streams 4 --batch 256" "--streams 3 --batch 1024" "--streams 2 --batch 1024"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 200 python -u bench.py --cpu-seconds 0 --no-profile --steps 8 $cfg > gpurun_out/sweep/$tag.log 2>&1
  echo "$cfg $(tail -1 gpurun_out/sweep/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
