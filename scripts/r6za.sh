#!/bin/bash
# Round 6: C1's first run on fresh engines in a warm process, plan modes 0 / 2 (+ KLF_DIAG marks)
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6za; mkdir -p $o
timeout -k 10 200 python3 scripts/cold_probe.py c1 > $o/cold.txt 2> $o/cold.err
KLF_DIAG=1 timeout -k 10 200 python3 scripts/cold_probe.py c1 > $o/cold_diag.txt 2> $o/cold_diag.err
cat $o/cold.txt
echo "r6za done"
