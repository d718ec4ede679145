#!/bin/bash
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6d; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
bash scripts/ab.sh $o/ab c5 2 base inl0:klogs_amd/_lib_inl0 > $o/ab_c5.txt 2>&1
bash scripts/ktrace_ab.sh $o c5 base > $o/kt_c5.txt 2>&1
bash scripts/ktrace_ab.sh $o c2 base > $o/kt_c2.txt 2>&1
bash scripts/ktrace_ab.sh $o c1 base > $o/kt_c1.txt 2>&1
echo "r6d done"
