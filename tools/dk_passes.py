"""Durand-Kerner f64 issue per pass.

Each merged RANSAC round (one per pipelined submit: every pending batch takes its next round,
csrc/geometry.hip launch_round) launches ransac_dk_kernel three times, passes 0, 1, 2 (48 / 80 /
the remaining sweeps).  From the raw rocprofv3
--pmc counter_collection.csv of the f64 pass (tools/pmc_stall_f64.sh: SQ_INSTS_VALU_*_F64,
SQ_WAVES, SQ_WAVE_CYCLES per dispatch) and the kernel-trace CSV of the same short bench
without counters (per-dispatch start / end), per (round, pass): mean f64 wave-instructions,
waves, duration, and the issue fraction = f64 wave-instructions x 4 cycles (a wave64 f64 op on
a 16-lane f64 pipe) / (duration x 2.4 GHz x 1024 SIMDs).

With the lane pass's raw counter CSV (SQ_THREAD_CYCLES_VALU, SQ_ACTIVE_INST_VALU per dispatch),
each pass's VALU lane utilisation and its issue fraction weighted by it.

usage: python tools/dk_passes.py <counter_collection.csv> <kernel_trace.csv> <out.json> [lanes.csv]"""
import collections
import csv
import json
import os
import sys

F64 = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")
CLOCK_HZ, SIMDS, CYCLES_PER_F64 = 2.4e9, 1024, 4
PASSES = 3


def _dk(name):
    return "ransac_dk_kernel" in (name or "")


def _per_dispatch(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if _dk(r.get("Kernel_Name")):
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def main(pmc_csv, trace_csv, dst, lanes_csv=None):
    pmc = _per_dispatch(pmc_csv)
    lanes = _per_dispatch(lanes_csv) if lanes_csv and os.path.exists(lanes_csv) else []
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            for r in sorted((r for r in csv.DictReader(open(trace_csv)) if _dk(r.get("Kernel_Name"))),
                            key=lambda r: int(r["Dispatch_Id"]))]
    rows = []
    for slot in range(PASSES):
        c = pmc[slot::PASSES]
        d = durs[slot::PASSES]
        ln = lanes[slot::PASSES]
        if not c:
            continue
        f64 = sum(sum(x.get(k, 0.0) for k in F64) for x in c) / len(c)
        waves = sum(x.get("SQ_WAVES", 0.0) for x in c) / len(c)
        dur = sum(d) / len(d) if d else None
        act = sum(x.get("SQ_ACTIVE_INST_VALU", 0.0) for x in ln)
        util = sum(x.get("SQ_THREAD_CYCLES_VALU", 0.0) for x in ln) / (64.0 * act) if act > 0 else None
        issue = f64 * CYCLES_PER_F64 / (dur * CLOCK_HZ * SIMDS) if dur else None
        rows.append({"pass": slot, "dispatches": len(c), "f64_wave_insts": f64,
                     "waves": waves, "ms": dur * 1e3 if dur else None, "issue_frac": issue,
                     "valu_lane_util": util, "issue_frac_lane_weighted": issue * util if issue and util else None})
    doc = {"source": "rocprofv3 --pmc (f64 pass, lane pass) and --kernel-trace of the same bench "
                     "(tools/profile_final.sh)",
           "tree": json.loads(os.environ["DVO_PMC_TREE"]) if os.environ.get("DVO_PMC_TREE") else None,
           "note": "issue_frac: f64 wave-instructions x 4 cycles / (kernel time x 2.4 GHz x 1024 SIMDs), issued "
                   "lane slots; valu_lane_util: SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64); "
                   "issue_frac_lane_weighted = issue_frac x valu_lane_util",
           "passes": rows}
    json.dump(doc, open(dst, "w"), indent=1)
    for r in rows:
        ms = f"{r['ms']:.3f}" if r["ms"] else "-"
        fr = f"{r['issue_frac']:.3f}" if r["issue_frac"] else "-"
        lu = f"{r['valu_lane_util']:.3f}" if r["valu_lane_util"] else "-"
        print(f"pass {r['pass']}: f64 wave-insts {r['f64_wave_insts']:.4g} waves {r['waves']:.0f} "
              f"ms {ms} issue {fr} lane util {lu}")


if __name__ == "__main__":
    main(*sys.argv[1:])
