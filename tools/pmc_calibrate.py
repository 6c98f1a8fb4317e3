"""FETCH_SIZE / WRITE_SIZE calibration factors per access width, from the
known-bytes kernels of tools/calib/pmc_calib.cpp (MI355X_MICROARCH.md §HBM:
only 16 B/lane streaming accesses are calibrated there).

usage: python tools/pmc_calibrate.py <calib_stdout.jsonl> <fetch.csv> <write.csv> <out.json>
factor = algorithmic bytes / counter bytes (multiply a reading by it)."""
import csv
import json
import sys


def load(path, counter):
    return {r["kernel"]: float(r[counter]) * 1024.0 for r in csv.DictReader(open(path)) if counter in r}


def rdreq_bytes(r):
    """Bytes of one kernel's read requests by size (gfx950 TCC_EA0_RDREQ_*B)."""
    return (32 * r.get("TCC_EA0_RDREQ_32B_sum", 0.0) + 64 * r.get("TCC_EA0_RDREQ_64B_sum", 0.0)
            + 128 * r.get("TCC_EA0_RDREQ_128B_sum", 0.0))


def main(known_path, fetch, write, dst, rdreq=None):
    known = {}
    for line in open(known_path):
        line = line.strip()
        if line.startswith("{"):
            d = json.loads(line)
            known[d["kernel"]] = d
    f, w = load(fetch, "FETCH_SIZE"), load(write, "WRITE_SIZE")
    out = {"unit": "factor = known bytes / counter bytes (rocprofv3 KB x 1024)", "read": {}, "write": {}}
    for k, d in sorted(known.items()):
        width = k.split("_", 2)[2]  # b32_buffer, b128_global, ...
        if "read_bytes" in d and k in f:
            out["read"][width] = {"known": d["read_bytes"], "fetch_size": f[k], "factor": d["read_bytes"] / f[k]}
        if "write_bytes" in d and k in w:
            out["write"][width] = {"known": d["write_bytes"], "write_size": w[k], "factor": d["write_bytes"] / w[k]}
    if rdreq:
        # the request-size decomposition the per-kernel traffic uses (pmc_traffic.py): factor ~1 expected
        rq = {r["kernel"]: {c: float(v) for c, v in r.items() if c.startswith("TCC_")} for r in csv.DictReader(open(rdreq))}
        out["read_requests"] = {}
        for k, d in sorted(known.items()):
            if "read_bytes" in d and k in rq:
                b = rdreq_bytes(rq[k])
                out["read_requests"][k.split("_", 2)[2]] = {
                    "known": d["read_bytes"], "request_bytes": b, "factor": d["read_bytes"] / b if b else None,
                    "requests": rq[k]}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
