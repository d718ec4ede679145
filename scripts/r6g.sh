#!/bin/bash
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6g; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
bash scripts/ab.sh $o/ab c3 2 pool 'rec::KLF_WAVE_POOL=0' > $o/ab_c3.txt 2>&1
bash scripts/ab.sh $o/ab c2 2 pool 'rec::KLF_WAVE_POOL=0' > $o/ab_c2.txt 2>&1
bash scripts/ab.sh $o/ab c4 1 pool 'rec::KLF_WAVE_POOL=0' > $o/ab_c4.txt 2>&1
bash scripts/ab.sh $o/ab c5 1 pool 'rec::KLF_WAVE_POOL=0' > $o/ab_c5.txt 2>&1
bash scripts/ktrace_ab.sh $o c5 base abl32:klogs_amd/_lib_abl32 > $o/kt_c5.txt 2>&1
KLF_DIAG=1 timeout -k 10 200 python3 scripts/run_config.py c5 --steps 2 > $o/diag_c5.json 2> $o/diag_c5.err
echo "r6g done"
