#!/bin/bash
# fused-compaction tests, then C3 fused-scan phase timings (claimed vs round-robin turns)
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_compaction.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
tail -1 $out/pytest.log
for v in fdiag fstat; do
  KLF_DIAG=1 KLF_LIB_DIR=klogs_amd/_lib_$v timeout -k 10 240 python3 scripts/run_config.py c3 --steps 3 > $out/c3_$v.json 2> $out/c3_$v.err
  grep "fused turns" $out/c3_$v.err | tail -1
  python3 -c "import json; d=json.load(open('$out/c3_$v.json')); print('$v', d['roofline']['avg_launch_ms'], d['device_ms_per_step'])"
done
timeout -k 10 240 python3 scripts/run_config.py c3 --steps 5 > $out/c3.json 2> $out/c3.err
python3 -c "import json; d=json.load(open('$out/c3.json')); print('c3', d['roofline']['avg_launch_ms'], d['device_ms_per_step'])"
echo done
