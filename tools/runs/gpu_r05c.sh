set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/trace_run.sh r05c_one_stream --streams 1 --steps 3 --warmup 1 &&
bash tools/trace_run.sh r05c_two_stream_tail --steps 6 --warmup 2 --tail-world 8
