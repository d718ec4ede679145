#!/bin/bash
# Round 6: plan modes A/B on C1 / C2 / C5 (same box)
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6t; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "plan_modes or graph_replay or c4_literal or windowed" -x -q --timeout 120 --timeout-method thread > $o/pytest_new.log 2>&1
tail -1 $o/pytest_new.log
bash scripts/ktrace_ab.sh $o c2 new old::KLF_PLAN_MODE=0 new2 > $o/kt_c2.txt 2>&1
bash scripts/ktrace_ab.sh $o c5 new old::KLF_PLAN_MODE=0 > $o/kt_c5.txt 2>&1
bash scripts/ktrace_ab.sh $o c1 new old::KLF_PLAN_MODE=0 one::KLF_PLAN_MODE=1 > $o/kt_c1.txt 2>&1
for c in c1 c2; do
  timeout -k 10 120 python scripts/run_config.py $c --steps 50 --warmup 5 > $o/${c}_new.json 2> $o/${c}_new.err
  KLF_PLAN_MODE=0 timeout -k 10 120 python scripts/run_config.py $c --steps 50 --warmup 5 > $o/${c}_old.json 2> $o/${c}_old.err
  timeout -k 10 120 python scripts/run_config.py $c --steps 50 --warmup 5 > $o/${c}_new2.json 2> $o/${c}_new2.err
done
echo "r6t done"
