"""Kernel sequence of the last batch in a single-stream rocprofv3 kernel trace:
each dvo:: launch with its start offset, duration and the idle gap before it.

usage: python tools/trace_sequence.py <kernel_trace.csv> [out.txt]"""
import csv
import sys


def main(src, dst=None):
    rows = []
    for r in csv.DictReader(open(src)):
        name = r.get("Kernel_Name", "")
        if "dvo::" not in name:
            continue
        k = name.replace("(anonymous namespace)::", "").split("(")[0].replace("dvo::", "").replace("void ", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    # the last batch starts at the last resize launch of level 1 (first kernel of a batch)
    starts = [i for i, (_, _, k) in enumerate(rows) if k.startswith("resize_level")]
    first = starts[-7] if len(starts) >= 7 else 0
    seq = rows[first:]
    t0 = seq[0][0]
    lines, prev_end = [], t0
    tot = {}
    for s, e, k in seq:
        lines.append(f"{(s - t0) / 1e3:10.1f} us  +gap {(s - prev_end) / 1e3:7.1f}  dur {(e - s) / 1e3:9.1f}  {k}")
        tot[k] = tot.get(k, 0) + (e - s) / 1e3
        prev_end = max(prev_end, e)
    lines.append(f"batch wall {(prev_end - t0) / 1e3:.1f} us")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        lines.append(f"  {k:28s} {v:9.1f} us")
    out = "\n".join(lines)
    print(out)
    if dst:
        open(dst, "w").write(out + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
