#!/bin/bash
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6c; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
bash scripts/ktrace_ab.sh $o c5 base abl16:klogs_amd/_lib_abl16 abl32768:klogs_amd/_lib_abl32768 > $o/kt_c5.txt 2>&1
bash scripts/ktrace_ab.sh $o c2 base abl1024:klogs_amd/_lib_abl1024 > $o/kt_c2.txt 2>&1
bash scripts/ab.sh $o/ab c3 1 base cua0:klogs_amd/_lib_cua0 > $o/ab_c3.txt 2>&1
bash scripts/ktrace_ab.sh $o c4 base > $o/kt_c4.txt 2>&1
KLF_DIAG=1 timeout -k 10 200 python3 scripts/run_config.py c2 --steps 3 > $o/diag_c2.json 2> $o/diag_c2.err
echo "r6c done"
