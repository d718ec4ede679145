#!/bin/bash
# Round-6 diagnostics on one GPU box (each step its own time limit, chained):
#   the -m gpu suite, kernel traces of C5 / C1 / C2, and the cold-run marks of C2.
#     bash scripts/r6_diag.sh OUT
set -e
cd "$(dirname "$0")/.."
out=$1
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -1 $out/pytest_gpu.log
bash scripts/trace_configs.sh "$out" c5 c1 c2
KLF_DIAG=1 timeout -k 10 300 python scripts/cold_diag.py c2 > $out/cold_c2.out 2> $out/cold_c2.err
echo "r6_diag done: $out"
