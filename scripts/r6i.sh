#!/bin/bash
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6i; mkdir -p $o
KLF_DIAG=1 KLF_DIAG_ALLOC=1 timeout -k 10 300 python scripts/cold_diag.py c5 > $o/cold_c5.out 2> $o/cold_c5.err
KLF_DIAG=1 KLF_DIAG_ALLOC=1 timeout -k 10 200 python scripts/cold_diag.py c1 > $o/cold_c1.out 2> $o/cold_c1.err
bash scripts/ktrace_ab.sh $o c5 base nofwd:klogs_amd/_lib_nofwd noback:klogs_amd/_lib_noback > $o/kt_c5.txt 2>&1
echo "r6i done"
