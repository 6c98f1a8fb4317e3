#!/bin/bash
# A/B of float k-NN variants (lib/exp/libdvo_<tag>.so): parity tests on the
# default build, then per-variant kernel durations from rocprofv3 --stats.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 120 python3 -u -m pytest tests/test_knn_float.py -x -q --timeout 60 --timeout-method thread -m gpu > gpurun_out/knn_ab_tests.log 2>&1
for v in base "$@"; do
  if [ "$v" = base ]; then unset DVO_LIB_PATH; else export DVO_LIB_PATH=$PWD/droplet_visual_odometry_amd/lib/exp/libdvo_$v.so; fi
  timeout -k 10 100 rocprofv3 --kernel-trace --stats -d /tmp/knn_$v -o run --output-format csv -- python3 tools/bench_knn.py > gpurun_out/knn_ab_$v.log 2>&1
  python3 - "$v" $(find /tmp/knn_$v -name "*kernel_stats.csv") >> gpurun_out/knn_ab.txt <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[2])):
    if "knn" in r["Name"]:
        print(sys.argv[1], r["Name"].replace("(anonymous namespace)::", "").split("(")[0][-48:], r["Calls"], "avg_us=%.1f min_us=%.1f max_us=%.1f" % (
            float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
PY
done
