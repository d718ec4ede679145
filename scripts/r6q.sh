#!/bin/bash
# Round 6: graph replay for small batches + one readback copy -- parity, then C1 / C2 steps
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6q; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
for c in c1 c2; do
  timeout -k 10 120 python scripts/run_config.py $c --steps 50 --warmup 5 > $o/${c}_graph.json 2> $o/${c}_graph.err
  KLF_GRAPH=0 timeout -k 10 120 python scripts/run_config.py $c --steps 50 --warmup 5 > $o/${c}_eager.json 2> $o/${c}_eager.err
done
KLF_DIAG=1 timeout -k 10 120 python scripts/run_config.py c1 --steps 10 --warmup 3 > $o/c1_diag.json 2> $o/c1_diag.err
bash scripts/ktrace_ab.sh $o c1 graph eager::KLF_GRAPH=0 > $o/kt_c1.txt 2>&1
echo "r6q done"
