#!/bin/bash
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pattern_counts.py tests/test_gpu_tindex.py tests/test_gpu_large.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
tail -1 $out/pytest.log
bash scripts/ab_lib.sh $out c4 klogs_amd/_lib_prev klogs_amd/_lib 1
bash scripts/ab_lib.sh $out c5 klogs_amd/_lib_prev klogs_amd/_lib 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/tr_c4 -o run -- python3 scripts/run_config.py c4 --steps 3 > $out/tr_c4.json 2> $out/tr_c4.err
echo done
