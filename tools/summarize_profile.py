"""Filter a rocprofv3 --stats kernel CSV down to the libdvo_hip kernels.

usage: python tools/summarize_profile.py <run_kernel_stats.csv> <out.csv> [steps]
Writes the dvo:: rows (the product kernels; torch's synthetic-frame rendering is
input setup outside the timed region) and prints a per-kernel table.
"""
import csv
import sys


def main(src, dst, steps=None):
    rows = [r for r in csv.DictReader(open(src)) if "dvo::" in r["Name"]]
    with open(dst, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        for r in rows:
            w.writerow(r)
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    for r in rows:
        name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("dvo::", "")
        print(f"{name:28s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs'])/1e3:10.1f} "
              f"share={100*float(r['TotalDurationNs'])/tot:5.1f}%")


if __name__ == "__main__":
    main(*sys.argv[1:])
