#!/bin/bash
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6j; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
timeout -k 10 700 python bench.py > $o/bench.json 2> $o/bench.err
echo "r6j done"
