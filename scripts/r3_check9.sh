#!/bin/bash
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_compaction.py tests/test_gpu_fused.py tests/test_gpu_split.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
tail -1 $out/pytest.log
KLF_DIAG=1 timeout -k 10 200 python3 scripts/run_config.py c3 --steps 2 2>&1 >/dev/null | grep "k_tcopy" | head -1
bash scripts/ab_lib.sh $out c3 klogs_amd/_lib_prev klogs_amd/_lib 2
