#!/bin/bash
# Round 6: C1's latency -- per-kernel trace and the host marks of steady runs (KLF_DIAG)
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6n; mkdir -p $o
bash scripts/ktrace_ab.sh $o c1 base > $o/kt_c1.txt 2>&1
bash scripts/ktrace_ab.sh $o c2 base > $o/kt_c2.txt 2>&1
KLF_DIAG=1 timeout -k 10 120 python scripts/run_config.py c1 --steps 20 --warmup 3 > $o/c1_diag.json 2> $o/c1_diag.err
python3 - <<'P' > $o/c1_trace_gaps.txt
import csv, glob
f = sorted(glob.glob("gpurun_out/r6n/t_c1_base/**/run_kernel_trace.csv", recursive=True))[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
prev = None
for r in rows[-40:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0
    print(f"{r['Kernel_Name'][:40]:40s} gap {gap:8.2f} us  dur {(e - s) / 1e3:8.2f} us")
    prev = e
P
echo "r6n done"
