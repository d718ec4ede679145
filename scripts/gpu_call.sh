#!/bin/bash
# One GPU-box call: the -m gpu suite, smoke(), then a plain bench run (each step time-limited).
#     bash scripts/gpu_call.sh OUTDIR [bench args...]
set -e
O=$1; shift
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err
echo "gpu_call done: $O"
