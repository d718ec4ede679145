#!/bin/bash
# GPU tests, then C4 / C5 traces and their prefilter hit counts (KLF_DIAG).
set -e
cd "$(dirname "$0")/.."
out=$1
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -1 $out/pytest_gpu.log
for c in c4 c5; do
  KLF_DIAG=1 timeout -k 10 200 python3 scripts/run_config.py $c --steps 1 --warmup 0 > $out/diag_$c.json 2> $out/diag_$c.err
done
bash scripts/trace_configs.sh $out c4 c5
