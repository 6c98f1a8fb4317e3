"""Merge the FETCH_SIZE and WRITE_SIZE pass summaries (tools/pmc_summary.py
output) into the per-launch HBM traffic file bench.py reads for roofline.traffic.

usage: python tools/pmc_traffic.py <fetch.csv> <write.csv> <out.json> [batch]
rocprofv3 reports both counters in KB; x1024 is applied. The default bench
configuration (1280x720, 2000 features, the given batch (default 1024), one
stream) is recorded."""
import csv
import json
import sys


def load(path, counter):
    return {r["kernel"]: float(r[counter]) * 1024.0 for r in csv.DictReader(open(path)) if counter in r}


def main(fetch, write, dst, batch=1024):
    f, w = load(fetch, "FETCH_SIZE"), load(write, "WRITE_SIZE")
    doc = {
        "config": {"width": 1280, "height": 720, "nfeatures": 2000, "batch": int(batch), "streams": 1},
        "unit": "bytes per launch (rocprofv3 FETCH_SIZE/WRITE_SIZE are KB; x1024 applied)",
        "note": "separate --pmc passes (FETCH_SIZE, WRITE_SIZE), mean over dispatches; the byte kernels "
                "load 4-16 B/lane, for which the guide's x2 FETCH_SIZE correction (16 B/lane streaming reads) "
                "is not calibrated, so the raw value is reported",
        "kernels": {k: {"fetch_bytes": f.get(k, 0.0), "write_bytes": w.get(k, 0.0)} for k in sorted(set(f) | set(w))},
    }
    json.dump(doc, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
