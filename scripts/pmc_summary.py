#!/usr/bin/env python3
"""Per-kernel means of the counters in the passes scripts/pmc.sh wrote:
    python scripts/pmc_summary.py OUTDIR [--json out.json]
Rows of one dispatch (rocprofv3 may report a counter per hardware instance) are summed, then
averaged over the kernel's dispatches.  FETCH_SIZE is doubled (gfx950 wide streaming reads,
MI355X_MICROARCH.md HBM section) and both sizes are reported in bytes; SQ_* cycle counters
are as collected."""
import collections
import csv
import glob
import json
import re
import sys

# kernel -> counter -> dispatch -> summed value
agg = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for f in sorted(glob.glob(sys.argv[1] + "/*/p_counter_collection.csv")):
    for i, r in enumerate(csv.DictReader(open(f))):
        k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("klf::(anonymous namespace)::", "").replace("void ", ""))
        disp = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(i)
        agg[k][r["Counter_Name"]][(f, disp)] += float(r["Counter_Value"])
res = {}
for k, d in sorted(agg.items()):
    row = {c: sum(v.values()) / len(v) for c, v in d.items()}
    row["dispatches"] = max(len(v) for v in d.values())
    if "FETCH_SIZE" in row:
        row["fetch_bytes_x2"] = 2 * 1024 * row.pop("FETCH_SIZE")
    if "WRITE_SIZE" in row:
        row["write_bytes"] = 1024 * row.pop("WRITE_SIZE")
    res[k] = row
    print(k, {c: "%.4g" % v for c, v in sorted(row.items())})
if "--json" in sys.argv:
    json.dump(res, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
