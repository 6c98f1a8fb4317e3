"""Per-launch f64 VALU instruction counts of every kernel from the f64 PMC pass
(tools/pmc_stall_f64.sh: SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64 over a short
one-stream bench, `launches` batch launches of `batch` new frames), as the JSON
bench.py prices its RANSAC f64-issue fraction from.

usage: python tools/pmc_f64.py <pmc_f64.csv> <out.json> [batch=512] [launches=2] [width height nfeatures]

DVO_PMC_LANES: the lane pass's summary (SQ_THREAD_CYCLES_VALU, SQ_ACTIVE_INST_VALU per kernel,
tools/profile_final.sh): each kernel's VALU lane utilisation, THREAD_CYCLES / (ACTIVE_INST x 64)
(rocprofv3's VALUUtilization), and its f64 FLOPs weighted by it.  The utilisation is over all of
the kernel's VALU instructions, the f64 ones among them.  DVO_PMC_TREE / DVO_PMC_STREAMS: the
profiled tree and stream count, copied into the document."""
import csv
import json
import os
import sys

F64 = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")


def main(src, dst, batch=512, launches=2, width=1280, height=720, nfeatures=2000):
    batch, launches = int(batch), int(launches)
    kernels = {}
    rows = list(csv.DictReader(open(src)))
    # launches: normalize_kernel runs once per batch launch (falls back to the argument)
    launches = next((int(r["dispatches"]) for r in rows if r["kernel"] == "normalize_kernel"), launches)
    for r in rows:
        d = int(r["dispatches"])
        per = d / launches  # dispatches per batch launch; the CSV holds means per dispatch
        k = {c.replace("SQ_INSTS_VALU_", "").lower(): float(r.get(c) or 0.0) * per for c in F64}
        k["valu"] = float(r.get("SQ_INSTS_VALU") or 0.0) * per
        k["waves"] = float(r.get("SQ_WAVES") or 0.0) * per
        k["dispatches_per_launch"] = per
        # wave64 f64 FLOPs if every lane were active: FMA = 2, others 1
        k["f64_wave_insts"] = sum(k[c] for c in ("fma_f64", "mul_f64", "add_f64", "trans_f64"))
        k["f64_flops_full_wave"] = 64.0 * (2 * k["fma_f64"] + k["mul_f64"] + k["add_f64"] + k["trans_f64"])
        kernels[r["kernel"]] = k
    lanes = os.environ.get("DVO_PMC_LANES")
    if lanes and os.path.exists(lanes):
        for r in csv.DictReader(open(lanes)):
            k = kernels.get(r["kernel"])
            act = float(r.get("SQ_ACTIVE_INST_VALU") or 0.0)
            if k is None or act <= 0:
                continue
            u = float(r.get("SQ_THREAD_CYCLES_VALU") or 0.0) / (act * 64.0)
            k["valu_lane_util"] = u
            k["f64_flops_lane_weighted"] = k["f64_flops_full_wave"] * u
    doc = {"config": {"width": int(width), "height": int(height), "nfeatures": int(nfeatures), "batch": batch,
                      "launches": launches, "streams": int(os.environ.get("DVO_PMC_STREAMS", "1"))},
           "tree": json.loads(os.environ["DVO_PMC_TREE"]) if os.environ.get("DVO_PMC_TREE") else None,
           "source": "rocprofv3 --pmc SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64 SQ_INSTS_VALU SQ_WAVES (tools/pmc_stall_f64.sh)",
           "kernels": kernels}
    json.dump(doc, open(dst, "w"), indent=1)
    for n, k in sorted(kernels.items(), key=lambda x: -x[1]["f64_wave_insts"])[:12]:
        print(f"{n:40s} f64 wave-insts/launch {k['f64_wave_insts']:.4g}  valu {k['valu']:.4g}  "
              f"lane util {k.get('valu_lane_util', float('nan')):.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
