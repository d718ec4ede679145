#!/bin/bash
# Parity + C5 A/B of the probe-fold-variants branch build (klogs_amd/_lib_var) against main (_lib).
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
export TMPDIR=/tmp
KLF_LIB_DIR=klogs_amd/_lib_var timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pattern_counts.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
tail -1 $out/pytest.log
bash scripts/ab_lib.sh $out c5 klogs_amd/_lib klogs_amd/_lib_var 2
