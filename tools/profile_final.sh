#!/bin/bash
# End-of-round profile at the bench's own configuration (batch 3072, two streams, the pipelined
# RANSAC rounds), in two GPU parts (each fits one gpurun call) and a merge that runs anywhere:
#   a  rocprofv3 --kernel-trace --stats of the default bench (side legs off), then the
#      FETCH_SIZE and WRITE_SIZE passes over the same bench at one timed step, each beside the
#      known-bytes calibration kernels (tools/calib);
#   b (= b1 + b2)  b1: the read-request-size pass (+ calibration), the SQ instruction pass, the stall pass, the
#      f64 pass, the lane pass (SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU: active lanes per VALU
#      instruction) and a counter-free kernel trace for the Durand-Kerner per-pass durations;
#   merge  -> gpurun_out/prof/<tag>_{pmc_traffic,pmc_f64,dk_passes}.json, each carrying the tree
#      (DVO_TREE, the git commit, passed in by the caller) and the library's source hash.
# Counter passes collect on the library's kernels only (--kernel-include-regex dvo::): the synthetic
# frames are rendered by torch kernels, which counter collection would serialise one by one.
# Every counter pass runs the bench with its timed step, priming and drain: per-launch figures are
# the run's totals over its batch launches (normalize_kernel dispatches), so the pipeline's ramp
# and drain rounds are counted with the batches they belong to.
# usage: DVO_TREE=<commit> tools/profile_final.sh TAG a|b|merge
set -e
tag=$1; part=$2; shift 2
root=$(pwd)
out="$root/gpurun_out/prof"
mkdir -p "$out"
B=${B:-3072}
S=${S:-2}
SP=${SP:-1}  # the counter passes: one stream (rocprofv3 --pmc serialises dispatches; with two streams their cross-stream waits stalled it)
side="--cpu-seconds 0 --no-ref-equivalent --no-host-fed --tail-world 0 --dropin-seconds 0 --pose-check-32 0 --config-legs none"
pass="$WL --batch $B --streams $SP --steps 1 --warmup 1 --runs 1 --no-profile $side"
tree="{\"git\": \"${DVO_TREE:-unknown}\", \"source_hash\": \"$(cd "$root" && python3 -c 'from droplet_visual_odometry_amd.build import source_hash; print(source_hash())')\"}"
if [ "$part" = merge ]; then
  python3 "$root/tools/pmc_calibrate.py" "$out/${tag}_calib_known.jsonl" "$out/${tag}_calib_FETCH_SIZE.csv" "$out/${tag}_calib_WRITE_SIZE.csv" "$out/${tag}_pmc_calibration.json" "$out/${tag}_calib_rdreq.csv" > /dev/null
  DVO_PMC_TREE="$tree" DVO_PMC_STREAMS=$SP python3 "$root/tools/pmc_traffic.py" "$out/${tag}_pmc_FETCH_SIZE.csv" "$out/${tag}_pmc_WRITE_SIZE.csv" "$out/${tag}_pmc_sq.csv" "$out/${tag}_pmc_calibration.json" "$out/${tag}_pmc_traffic.json" $B "$out/${tag}_pmc_rdreq.csv"
  DVO_PMC_TREE="$tree" DVO_PMC_STREAMS=$SP DVO_PMC_LANES="$out/${tag}_pmc_lanes.csv" python3 "$root/tools/pmc_f64.py" "$out/${tag}_pmc_f64.csv" "$out/${tag}_pmc_f64.json" $B
  DVO_PMC_TREE="$tree" python3 "$root/tools/dk_passes.py" "$out/${tag}_f64_raw.csv" "$out/${tag}_kt_raw.csv" "$out/${tag}_dk_passes.json" "$out/${tag}_lanes_raw.csv" > "$out/${tag}_dk_passes.txt"
  exit 0
fi
export TMPDIR=/tmp
cd /tmp
run_pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 170 rocprofv3 --pmc "$@" --kernel-include-regex 'dvo::' -d /tmp/pmc_${tag}_$name -o run --output-format csv -- python3 "$root/bench.py" $pass > "$out/${tag}_pmc_$name.log" 2>&1
  python3 "$root/tools/pmc_summary.py" $(find /tmp/pmc_${tag}_$name -name '*counter_collection.csv') "$out/${tag}_pmc_$name.csv" > /dev/null
}
calib_pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 60 rocprofv3 --pmc "$@" -d /tmp/cal_${tag}_$name -o run --output-format csv -- "$root/tools/calib/build/pmc_calib" > "$out/${tag}_calib_known.jsonl" 2> "$out/${tag}_calib_$name.log"
  python3 "$root/tools/pmc_summary.py" $(find /tmp/cal_${tag}_$name -name '*counter_collection.csv') "$out/${tag}_calib_$name.csv" > /dev/null
}
if [ "$part" = a ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/st_$tag -o run --output-format csv -- python3 "$root/bench.py" $WL $side > "$out/${tag}_bench_under_rocprof.log" 2>&1
  python3 "$root/tools/summarize_profile.py" $(find /tmp/st_$tag -name '*kernel_stats.csv') "$out/${tag}_kernel_stats.csv" > "$out/${tag}_kernel_stats.txt"
  for c in FETCH_SIZE WRITE_SIZE; do
    run_pass $c $c
    calib_pass $c $c
  done
fi
if [ "$part" = b ] || [ "$part" = b1 ]; then
  rq="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
  run_pass rdreq $rq
  calib_pass rdreq $rq
  run_pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
  run_pass stall SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
fi
if [ "$part" = b ] || [ "$part" = b2 ]; then
  run_pass f64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES
  awk 'NR == 1 || /ransac_dk_kernel/' $(find /tmp/pmc_${tag}_f64 -name '*counter_collection.csv') > "$out/${tag}_f64_raw.csv"
  run_pass lanes SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES
  awk 'NR == 1 || /ransac_dk_kernel/' $(find /tmp/pmc_${tag}_lanes -name '*counter_collection.csv') > "$out/${tag}_lanes_raw.csv"
  timeout -k 10 170 rocprofv3 --kernel-trace -d /tmp/pmc_${tag}_kt -o run --output-format csv -- python3 "$root/bench.py" $pass > "$out/${tag}_kt.log" 2>&1
  awk 'NR == 1 || /ransac_dk_kernel/' $(find /tmp/pmc_${tag}_kt -name '*kernel_trace.csv') > "$out/${tag}_kt_raw.csv"
fi
rm -rf /tmp/st_$tag /tmp/pmc_${tag}_* /tmp/cal_${tag}_*
