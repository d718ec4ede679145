#!/bin/bash
# Round 6: C1 / C2 step time with and without the scan's dispatch events (same box, alternating)
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6zc; mkdir -p $o
for i in 1 2; do
  for c in c1 c2; do
    timeout -k 10 120 python scripts/run_config.py $c --steps 200 --warmup 10 > $o/${c}_ev_$i.json 2> $o/${c}_ev_$i.err
    KLF_SCAN_EVENTS=0 timeout -k 10 120 python scripts/run_config.py $c --steps 200 --warmup 10 > $o/${c}_noev_$i.json 2> $o/${c}_noev_$i.err
  done
done
echo "r6zc done"
