#!/bin/bash
# Round 6: the line gather's copy chunks (k_cmove) -- chunk target 1024 / 2048 / 4096, U = 2 (C5, C2, C4 same box)
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6zb; mkdir -p $o
for c in c5 c2 c4; do
  bash scripts/ktrace_ab.sh $o $c base ct2k:klogs_amd/_lib_ct2k ct4k:klogs_amd/_lib_ct4k cu2:klogs_amd/_lib_cu2 > $o/kt_$c.txt 2>&1
done
echo "r6zb done"
