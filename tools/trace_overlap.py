"""Overlap of the two in-flight batches in a multi-stream rocprofv3 kernel trace.

For the window from the 2nd-to-last batch start to the end, every dvo:: kernel
gets its total duration and its "solo" time (when no other dvo:: kernel was
running, i.e. the time it held the GPU alone), plus the window's idle time.
Solo time is the part of a kernel the other stream did not hide.

usage: python tools/trace_overlap.py <kernel_trace.csv> [out.txt]"""
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
    # batch boundaries: the end of each batch's pose chain (its last kernel)
    ends = [e for _, e, k in rows if k.startswith("pose_chain")]
    t0, t1 = (ends[-4], ends[-1]) if len(ends) >= 4 else (rows[0][0], rows[-1][1])
    win = [(max(s, t0), min(e, t1), k) for s, e, k in rows if e > t0 and s < t1]
    # sweep over boundaries
    ev = sorted({t for s, e, _ in win for t in (s, e)} | {t0, t1})
    tot, solo = {}, {}
    idle = 0
    for s, e, k in win:
        tot[k] = tot.get(k, 0) + (e - s)
    for a, b in zip(ev, ev[1:]):
        live = [k for s, e, k in win if s <= a and e >= b]
        if not live:
            idle += b - a
        elif len(live) == 1:
            solo[live[0]] = solo.get(live[0], 0) + (b - a)
    wall = t1 - t0
    gaps = []
    busy_until = t0
    for s_, e_, _ in sorted(win):
        if s_ > busy_until + 20_000:  # idle stretches over 20 us
            gaps.append((busy_until - t0, s_ - busy_until))
        busy_until = max(busy_until, e_)
    lines = [f"window {wall / 1e3:.1f} us over 3 batches ({wall / 3e3:.1f} us per batch), idle {idle / 1e3:.1f} us",
             "idle stretches > 20 us (offset us, length us): " + ", ".join(f"({o / 1e3:.0f}, {g / 1e3:.0f})" for o, g in gaps),
             f"{'kernel':28s} {'total us':>10s} {'solo us':>10s}  (per batch)"]
    for k, v in sorted(tot.items(), key=lambda kv: -solo.get(kv[0], 0)):
        lines.append(f"{k:28s} {v / 3e3:10.1f} {solo.get(k, 0) / 3e3:10.1f}")
    out = "\n".join(lines)
    print(out)
    if dst:
        open(dst, "w").write(out + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
