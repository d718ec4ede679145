#!/bin/bash
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6f; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
bash scripts/ab.sh $o/ab c5 2 pool 'rec::KLF_WAVE_POOL=0' > $o/ab_c5.txt 2>&1
bash scripts/ab.sh $o/ab c4 1 pool 'rec::KLF_WAVE_POOL=0' > $o/ab_c4.txt 2>&1
bash scripts/ab.sh $o/ab c3 1 pool 'rec::KLF_WAVE_POOL=0' > $o/ab_c3.txt 2>&1
bash scripts/ab.sh $o/ab c2 1 pool 'rec::KLF_WAVE_POOL=0' > $o/ab_c2.txt 2>&1
echo "r6f done"
