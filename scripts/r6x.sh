#!/bin/bash
# Round 6: first-run cost breakdown (KLF_DIAG marks) of C1 / C2 / C5 cold engines
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6x; mkdir -p $o
for c in c1 c2 c5; do
  KLF_DIAG=1 timeout -k 10 200 python scripts/run_config.py $c --steps 2 --warmup 1 > $o/${c}.json 2> $o/${c}.err
done
echo "r6x done"
