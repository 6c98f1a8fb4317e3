"""Merge the PMC passes of a round profile into the per-launch file bench.py
reads for roofline.traffic and roofline.valu.

usage: python tools/pmc_traffic.py <fetch.csv> <write.csv> <sq.csv> <calibration.json> <out.json> [batch]

fetch/write: FETCH_SIZE / WRITE_SIZE passes (tools/pmc_summary.py output;
rocprofv3 reports KB, x1024 applied).  sq: the SQ_INSTS_* pass.  calibration:
tools/pmc_calibrate.py output; a kernel's readings are multiplied by the
factor of the access width it uses (KERNEL_WIDTHS, from the kernel source);
kernels not listed keep their raw readings (calibrated: false)."""
import csv
import json
import os
import sys

# (read width, write width) of the dominant accesses, per kernel (orb.hip)
KERNEL_WIDTHS = {
    "fast_strip_kernel": ("b32_buffer", "b32_global"),  # raw_buffer_load_b32 rows; 4-byte key / count stores
    "blur_kernel": ("b32_buffer", "b32_global"),        # raw_buffer_load_b32 rows; one word per lane and row
}


def load(path, counters):
    """Per kernel: its counters per batch launch = the mean per dispatch x dispatches per launch
    (a kernel can run several times per batch: pyramid levels, RANSAC rounds and passes, frame
    groups of the detection).  Launches = the dispatches of normalize_kernel (once per batch)."""
    rows = list(csv.DictReader(open(path)))
    launches = next((float(r["dispatches"]) for r in rows if r["kernel"] == "normalize_kernel"), 2.0)
    out = {}
    for r in rows:
        per = float(r.get("dispatches") or launches) / launches
        out[r["kernel"]] = {c: float(r[c]) * per for c in counters if c in r and r[c] != ""}
    return out


RQ = ["TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_sum"]


def main(fetch, write, sq, calib, dst, batch=1024, rdreq=None):
    f = load(fetch, ["FETCH_SIZE"])
    rq = load(rdreq, RQ) if rdreq else {}
    w = load(write, ["WRITE_SIZE"])
    s = load(sq, ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"])
    cal = json.load(open(calib))
    kernels = {}
    for k in sorted(set(f) | set(w) | set(s)):
        fr = f.get(k, {}).get("FETCH_SIZE", 0.0) * 1024.0
        wr = w.get(k, {}).get("WRITE_SIZE", 0.0) * 1024.0
        e = {"fetch_bytes_raw": fr, "write_bytes_raw": wr}
        if k in rq:
            # every kernel: the bytes of its read requests by size (32/64/128 B, gfx950 TCC_EA0_RDREQ_*B),
            # checked on the known-bytes kernels (calibration read_requests); writes: WRITE_SIZE, exact for
            # the calibrated store widths
            r = rq[k]
            fb = 32 * r.get(RQ[0], 0.0) + 64 * r.get(RQ[1], 0.0) + 128 * r.get(RQ[2], 0.0)
            e.update(fetch_bytes=fb, write_bytes=wr, calibrated=True,
                     widths={"read": "request sizes", "requests": r, "write": "WRITE_SIZE"})
        elif k in KERNEL_WIDTHS:
            rw, ww = KERNEL_WIDTHS[k]
            fa, wa = cal["read"][rw]["factor"], cal["write"][ww]["factor"]
            e.update(fetch_bytes=fr * fa, write_bytes=wr * wa, calibrated=True,
                     widths={"read": rw, "write": ww, "read_factor": fa, "write_factor": wa})
        else:
            e.update(fetch_bytes=fr, write_bytes=wr, calibrated=False)
        for c, v in s.get(k, {}).items():
            e[c] = v
        kernels[k] = e
    doc = {
        # the workload the passes ran (tools/profile_round.sh WL=...): DVO_PMC_CONFIG="width height nfeatures"
        "config": dict(zip(("width", "height", "nfeatures"),
                           (int(v) for v in os.environ.get("DVO_PMC_CONFIG", "1280 720 2000").split())),
                       batch=int(batch), streams=int(os.environ.get("DVO_PMC_STREAMS", "1"))),
        # the profiled tree (tools/profile_final.sh): git commit and the library's source hash
        "tree": json.loads(os.environ["DVO_PMC_TREE"]) if os.environ.get("DVO_PMC_TREE") else None,
        "unit": "per launch: bytes (FETCH_SIZE/WRITE_SIZE KB x1024, then the width calibration), "
                "SQ_* instruction counts (wave-level)",
        "note": "separate --pmc passes (FETCH_SIZE; WRITE_SIZE; SQ instruction counts); per batch launch: the "
                "mean over dispatches x dispatches per launch",
        "calibration": os.path.basename(calib),
        "read_bytes": "32 n32 + 64 n64 + 128 n128 from the TCC_EA0_RDREQ_*B pass" if rq else "FETCH_SIZE x width factor",
        "kernels": kernels,
    }
    json.dump(doc, open(dst, "w"), indent=1)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(*a[:5], int(a[5]) if len(a) > 5 else 1024, a[6] if len(a) > 6 else None)
