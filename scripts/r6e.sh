#!/bin/bash
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6e; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
bash scripts/ab.sh $o/ab c4 1 base hin0:klogs_amd/_lib_hin0 nrec:klogs_amd/_lib_nrec ntst:klogs_amd/_lib_ntst > $o/ab_c4.txt 2>&1
bash scripts/ab.sh $o/ab c5 1 base nrec:klogs_amd/_lib_nrec ntst:klogs_amd/_lib_ntst > $o/ab_c5.txt 2>&1
bash scripts/ktrace_ab.sh $o c4 base vpar0:klogs_amd/_lib_vpar0 > $o/kt_c4.txt 2>&1
echo "r6e done"
