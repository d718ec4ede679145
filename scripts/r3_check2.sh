#!/bin/bash
# GPU suite, then C3 fused-scan phase timings (dynamic vs round-robin turns) and C4/C5 scans.
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -1 $out/pytest_gpu.log
for v in fdiag fstat; do
  KLF_DIAG=1 KLF_LIB_DIR=klogs_amd/_lib_$v timeout -k 10 240 python3 scripts/run_config.py c3 --steps 3 > $out/c3_$v.json 2> $out/c3_$v.err
  grep "fused turns" $out/c3_$v.err | tail -2
done
for c in c5 c4; do
  timeout -k 10 240 python3 scripts/run_config.py $c --steps 5 > $out/$c.json 2> $out/$c.err
  python3 -c "import json; d=json.load(open('$out/$c.json')); print('$c', d['roofline']['avg_launch_ms'], d['device_ms_per_step'])"
done
echo done
