#!/usr/bin/env python3
"""Per-kernel means of the counters in the passes scripts/pmc.sh wrote:
    python scripts/pmc_summary.py OUTDIR [--json out.json]
FETCH_SIZE is doubled (gfx950 wide streaming reads, MI355X_MICROARCH.md HBM section) and
both sizes are reported in bytes; SQ_* cycle counters are quad-cycles as collected."""
import collections
import csv
import glob
import json
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("klf::(anonymous namespace)::", "").replace("void ", ""))
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k, d in sorted(agg.items()):
    row = {c: sum(v) / len(v) for c, v in d.items()}
    if "FETCH_SIZE" in row:
        row["fetch_bytes_x2"] = 2 * 1024 * row.pop("FETCH_SIZE")
    if "WRITE_SIZE" in row:
        row["write_bytes"] = 1024 * row.pop("WRITE_SIZE")
    res[k] = row
    print(k, {c: "%.4g" % v for c, v in sorted(row.items())})
if "--json" in sys.argv:
    json.dump(res, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
