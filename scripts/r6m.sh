#!/bin/bash
# Round 6: k_verify's bucket walk, entries loaded 4 / 2 / 1 at once (C4, C5 kernel traces)
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6m; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
bash scripts/ktrace_ab.sh $o c4 ent4 ent1:klogs_amd/_lib_ent1 ent2:klogs_amd/_lib_ent2 > $o/kt_c4.txt 2>&1
bash scripts/ktrace_ab.sh $o c5 ent4 ent1:klogs_amd/_lib_ent1 ent2:klogs_amd/_lib_ent2 > $o/kt_c5.txt 2>&1
echo "r6m done"
