#!/bin/bash
# Round 6: k_tindex at 4 waves per SIMD (C4, C5 same box) + the suite on the final build
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6y; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
bash scripts/ktrace_ab.sh $o c4 base tw4:klogs_amd/_lib_tw4 > $o/kt_c4.txt 2>&1
bash scripts/ktrace_ab.sh $o c5 base tw4:klogs_amd/_lib_tw4 > $o/kt_c5.txt 2>&1
echo "r6y done"
