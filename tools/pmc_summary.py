"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel (dvo:: and the calib_ kernels).

usage: python tools/pmc_summary.py <counter_collection.csv> [out.csv]
Prints, per kernel, the mean over dispatches of every collected counter."""
import collections
import csv
import sys


def main(src, dst=None):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(src)):
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
        if "dvo::" not in name and not name.startswith("calib_"):
            continue
        k = name.replace("(anonymous namespace)::", "").split("(")[0].replace("dvo::", "")
        did = r.get("Dispatch_Id") or r.get("Dispatch-Id")
        disp[k].add(did)
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    rows = []
    for k, cs in acc.items():
        n = max(1, len(disp[k]))
        rows.append({"kernel": k, "dispatches": n, **{c: v / n for c, v in cs.items()}})
    rows.sort(key=lambda r: -r.get("SQ_WAVE_CYCLES", r.get("FETCH_SIZE", 0)))
    cols = ["kernel", "dispatches"] + sorted({c for r in rows for c in r if c not in ("kernel", "dispatches")})
    for r in rows:
        print(" ".join(f"{c}={r.get(c, 0):.4g}" if c != "kernel" else f"{r[c]:24s}" for c in cols))
    if dst:
        with open(dst, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=cols)
            w.writeheader()
            w.writerows(rows)


if __name__ == "__main__":
    main(*sys.argv[1:])
