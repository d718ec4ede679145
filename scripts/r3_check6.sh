#!/bin/bash
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pattern_counts.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
tail -1 $out/pytest.log
bash scripts/ab_lib.sh $out c5 klogs_amd/_lib_prev klogs_amd/_lib 2
