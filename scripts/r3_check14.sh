#!/bin/bash
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_compaction.py tests/test_gpu_split.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
tail -1 $out/pytest.log
for c in c5 c2; do
  KLF_DIAG=1 timeout -k 10 240 python3 scripts/run_config.py $c --steps 3 > $out/$c.json 2> $out/$c.err
  grep -E "run [0-9.]+ us|grown" $out/$c.err | head -4
  python3 -c "import json; d=json.load(open('$out/$c.json')); print('$c', d['device_ms_per_step'], d['cold'])"
done
