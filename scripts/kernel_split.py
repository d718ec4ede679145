#!/usr/bin/env python3
"""Per-kernel mean duration (µs, first launch of each kernel dropped) of a rocprofv3
kernel trace:  python3 scripts/kernel_split.py <dir>/run_kernel_trace.csv"""
import collections
import csv
import re
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("klf::(anonymous namespace)::", ""))
    d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    w = v[1:] or v
    print(f"{n:34s} n={len(v):3d} mean={sum(w) / len(w):10.1f} min={min(v):10.1f}")
