#!/bin/bash
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6h; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
bash scripts/ktrace_ab.sh $o c5 base > $o/kt_c5.txt 2>&1
bash scripts/ktrace_ab.sh $o c1 base > $o/kt_c1.txt 2>&1
timeout -k 10 600 python bench.py > $o/bench.json 2> $o/bench.err
echo "r6h done"
