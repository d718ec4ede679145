#!/bin/bash
# Round 6: the gather's plan in k_tailw / k_cplan's last block (fewer launches) -- parity, C1 / C2 / C5
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6s; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "plan_modes or graph_replay" -x -v --timeout 120 --timeout-method thread > $o/pytest_new.log 2>&1
tail -1 $o/pytest_new.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
for c in c1 c2; do
  timeout -k 10 120 python scripts/run_config.py $c --steps 50 --warmup 5 > $o/${c}_new.json 2> $o/${c}_new.err
  KLF_PLAN_MODE=0 timeout -k 10 120 python scripts/run_config.py $c --steps 50 --warmup 5 > $o/${c}_old.json 2> $o/${c}_old.err
done
bash scripts/ktrace_ab.sh $o c1 new old::KLF_PLAN_MODE=0 > $o/kt_c1.txt 2>&1
bash scripts/ktrace_ab.sh $o c2 new old::KLF_PLAN_MODE=0 > $o/kt_c2.txt 2>&1
echo "r6s done"
