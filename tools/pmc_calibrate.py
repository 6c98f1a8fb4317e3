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


def main(known_path, fetch, write, dst):
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
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
