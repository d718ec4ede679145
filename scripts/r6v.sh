#!/bin/bash
# Round 6: k_tindex<R, 1> flattening 4 hits per thread at once (C4, C5 same box) + the suite
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6v; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
bash scripts/ktrace_ab.sh $o c4 fb4 fb1:klogs_amd/_lib_fb1 > $o/kt_c4.txt 2>&1
bash scripts/ktrace_ab.sh $o c5 fb4 fb1:klogs_amd/_lib_fb1 > $o/kt_c5.txt 2>&1
echo "r6v done"
