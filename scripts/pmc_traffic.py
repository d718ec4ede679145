"""Per-launch HBM traffic of the bench's dominant kernel from rocprofv3 --pmc passes.

Usage: python scripts/pmc_traffic.py <fetch counter csv> <write counter csv> <out.json>

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  gfx950 correction
(/opt/skills/guides/MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of
a 16-B-per-lane streaming read, so it is doubled; WRITE_SIZE is taken as is.  bench.py
reports fetch + write per launch as roofline.traffic and names this file as the source.
"""
import csv
import json
import sys

KERNEL = "k_scan<1, 1>"  # the literal variant: BASELINE config 2 (C2)


def per_launch(path, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and KERNEL in r["Kernel_Name"]]
    if not vals:
        raise SystemExit(f"no {counter} rows for {KERNEL} in {path}")
    return sum(vals) / len(vals) * 1024.0, len(vals)


fetch, nf = per_launch(sys.argv[1], "FETCH_SIZE")
write, nw = per_launch(sys.argv[2], "WRITE_SIZE")
out = {"kernel": KERNEL, "fetch_bytes": round(2.0 * fetch), "write_bytes": round(write),
       "traffic_bytes": round(2.0 * fetch + write), "launches": [nf, nw],
       "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), WRITE_SIZE x1; KiB -> B",
       "sources": [sys.argv[1], sys.argv[2]]}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out))
