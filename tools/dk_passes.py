"""Durand-Kerner f64 issue per pass.

Each batch launches ransac_dk_kernel six times: rounds 1 and 2 (64 hypotheses, the rest) x
passes 0, 1, 2 (48 / 80 / the remaining sweeps, csrc/geometry.hip).  From the raw rocprofv3
--pmc counter_collection.csv of the f64 pass (tools/pmc_stall_f64.sh: SQ_INSTS_VALU_*_F64,
SQ_WAVES, SQ_WAVE_CYCLES per dispatch) and the kernel-trace CSV of the same short bench
without counters (per-dispatch start / end), per (round, pass): mean f64 wave-instructions,
waves, duration, and the issue fraction = f64 wave-instructions x 4 cycles (a wave64 f64 op on
a 16-lane f64 pipe) / (duration x 2.4 GHz x 1024 SIMDs).

usage: python tools/dk_passes.py <counter_collection.csv> <kernel_trace.csv> <out.json>"""
import collections
import csv
import json
import sys

F64 = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")
CLOCK_HZ, SIMDS, CYCLES_PER_F64 = 2.4e9, 1024, 4


def _dk(name):
    return "ransac_dk_kernel" in (name or "")


def main(pmc_csv, trace_csv, dst):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(pmc_csv)):
        if _dk(r.get("Kernel_Name")):
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    pmc = [per[k] for k in sorted(per)]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            for r in sorted((r for r in csv.DictReader(open(trace_csv)) if _dk(r.get("Kernel_Name"))),
                            key=lambda r: int(r["Dispatch_Id"]))]
    rows = []
    for slot in range(6):
        c = pmc[slot::6]
        d = durs[slot::6]
        if not c:
            continue
        f64 = sum(sum(x.get(k, 0.0) for k in F64) for x in c) / len(c)
        waves = sum(x.get("SQ_WAVES", 0.0) for x in c) / len(c)
        dur = sum(d) / len(d) if d else None
        rows.append({"round": slot // 3 + 1, "pass": slot % 3, "dispatches": len(c), "f64_wave_insts": f64,
                     "waves": waves, "ms": dur * 1e3 if dur else None,
                     "issue_frac": f64 * CYCLES_PER_F64 / (dur * CLOCK_HZ * SIMDS) if dur else None})
    doc = {"source": "rocprofv3 --pmc (f64 pass) and --kernel-trace of the same short one-stream bench",
           "note": "issue_frac: f64 wave-instructions x 4 cycles / (kernel time x 2.4 GHz x 1024 SIMDs)",
           "passes": rows}
    json.dump(doc, open(dst, "w"), indent=1)
    for r in rows:
        ms = f"{r['ms']:.3f}" if r["ms"] else "-"
        fr = f"{r['issue_frac']:.3f}" if r["issue_frac"] else "-"
        print(f"round {r['round']} pass {r['pass']}: f64 wave-insts {r['f64_wave_insts']:.4g} waves {r['waves']:.0f} "
              f"ms {ms} issue {fr}")


if __name__ == "__main__":
    main(*sys.argv[1:])
