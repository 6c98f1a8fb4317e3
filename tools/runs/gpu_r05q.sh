# does a rocprofv3 --pmc pass over the bench complete with 4 HW queues (bench default 8)?
set -o pipefail
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r05q
side="--cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 --steps 1 --warmup 1 --runs 1 --no-profile --streams 1"
( time GPU_MAX_HW_QUEUES=4 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d /tmp/q4 -o run --output-format csv -- python3 $R/bench.py $side --batch 512 ) > $R/gpurun_out/r05q/q4_b512.log 2>&1 || exit 1
( time GPU_MAX_HW_QUEUES=4 timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE -d /tmp/q4b -o run --output-format csv -- python3 $R/bench.py $side --batch 3072 ) > $R/gpurun_out/r05q/q4_b3072.log 2>&1 || exit 1
ls -la $(find /tmp/q4 /tmp/q4b -name '*counter_collection.csv') > $R/gpurun_out/r05q/files.txt
