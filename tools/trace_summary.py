"""Per (kernel, grid) mean duration of the dvo:: kernels in a rocprofv3 kernel_trace.csv.

usage: python tools/trace_summary.py <kernel_trace.csv> [out.txt]"""
import collections
import csv
import sys


def main(src, dst=None):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(src)):
        name = r.get("Kernel_Name", "")
        if "dvo::" not in name:
            continue
        k = name.replace("(anonymous namespace)::", "").split("(")[0].replace("dvo::", "")
        grid = (r.get("Grid_Size_X") or r.get("Grid_Size", "")) + "x" + (r.get("Grid_Size_Y") or "") + "x" + (r.get("Grid_Size_Z") or "")
        acc[(k, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    lines = []
    for (k, g), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"{k:28s} grid={g:20s} n={len(v):4d} mean_ms={sum(v) / len(v):8.4f} total_ms={sum(v):9.3f}")
    out = "\n".join(lines)
    print(out)
    if dst:
        open(dst, "w").write(out + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
