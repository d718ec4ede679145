#!/bin/bash
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6l; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
KLF_LIB_DIR=klogs_amd/_lib_vtl timeout -k 10 300 python scripts/vtl.py c5 /tmp/vtl_c5.bin > $o/vtl_c5.txt 2> $o/vtl_c5.err
KLF_LIB_DIR=klogs_amd/_lib_vtl timeout -k 10 300 python scripts/vtl.py c4 /tmp/vtl_c4.bin > $o/vtl_c4.txt 2> $o/vtl_c4.err
bash scripts/ktrace_ab.sh $o c4 base > $o/kt_c4.txt 2>&1
bash scripts/ktrace_ab.sh $o c5 base > $o/kt_c5.txt 2>&1
echo "r6l done"
