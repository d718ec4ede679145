#!/bin/bash
# GPU suite, then C5 / C4 scans
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -1 $out/pytest_gpu.log
for c in c5 c4; do
  KLF_DIAG=1 timeout -k 10 240 python3 scripts/run_config.py $c --steps 5 > $out/$c.json 2> $out/$c.err
  grep "prefilter layout" $out/$c.err | head -1
  python3 -c "import json; d=json.load(open('$out/$c.json')); print('$c', d['roofline']['avg_launch_ms'], d['device_ms_per_step'], d.get('cold'))"
done
echo done
