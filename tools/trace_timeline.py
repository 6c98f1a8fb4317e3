"""Concurrency summary of a rocprofv3 kernel_trace.csv (dvo:: kernels only).

For the window between the first and last dvo kernel: the union of busy time,
and for each kernel name the time during which it was the ONLY dvo kernel
running (its exposed time).  usage: python tools/trace_timeline.py <csv> [out]"""
import collections
import csv
import sys


def main(src, dst=None):
    ev = []
    for r in csv.DictReader(open(src)):
        name = r.get("Kernel_Name", "")
        if "dvo::" not in name:
            continue
        k = name.replace("(anonymous namespace)::", "").split("(")[0].replace("dvo::", "")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    ev.sort()
    pts = []
    for s, e, k in ev:
        pts.append((s, 1, k))
        pts.append((e, -1, k))
    pts.sort(key=lambda p: (p[0], p[1]))
    active = collections.Counter()
    exposed = collections.Counter()
    total = collections.Counter()
    busy = 0
    conc = collections.Counter()
    last = pts[0][0]
    for t, d, k in pts:
        dt = t - last
        n = sum(active.values())
        if n > 0:
            busy += dt
            conc[min(n, 4)] += dt
            if n == 1:
                exposed[next(iter(+active))] += dt
            for kk, c in active.items():
                if c:
                    total[kk] += dt * c
        active[k] += d
        if active[k] == 0:
            del active[k]
        last = t
    span = pts[-1][0] - pts[0][0]
    lines = [f"span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(span - busy) / 1e6:.3f} ms",
             "concurrency: " + "  ".join(f"{n}:{v / 1e6:.3f}ms" for n, v in sorted(conc.items())),
             f"{'kernel':28s} {'sum_ms':>9s} {'exposed_ms':>10s}"]
    for k, v in sorted(total.items(), key=lambda kv: -kv[1]):
        lines.append(f"{k:28s} {v / 1e6:9.3f} {exposed[k] / 1e6:10.3f}")
    out = "\n".join(lines)
    print(out)
    if dst:
        open(dst, "w").write(out + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
