#!/bin/bash
# Round 6, final build: the suite, smoke(), the driver's bench command (no profiler)
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/${1:-r6w}; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
tail -1 $o/smoke.log
timeout -k 10 700 python bench.py > $o/bench.json 2> $o/bench.err
echo "r6w done"
