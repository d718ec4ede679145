#!/bin/bash
# compaction / split tests (the dense path without a run table), then the first-run cost
# breakdown of C5 (allocations, statistics, layout, uploads)
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_compaction.py tests/test_gpu_split.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
tail -1 $out/pytest.log
KLF_DIAG=1 KLF_DIAG_ALLOC=1 timeout -k 10 240 python3 scripts/run_config.py c5 --steps 2 > $out/c5.json 2> $out/c5.err
grep -E "klf\] (run|first-batch|alloc [0-9]{7,})" $out/c5.err | tail -24
python3 -c "import json; d=json.load(open('$out/c5.json')); print(d['cold'], d['device_ms_per_step'])"
