#!/bin/bash
# Round 6, final build: the suite, smoke(), C1 / C2 with and without timing events
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6zd; mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
tail -1 $o/smoke.log
timeout -k 10 200 python3 scripts/c1_notiming.py c1 > $o/notiming_c1.txt 2> $o/notiming_c1.err
timeout -k 10 200 python3 scripts/c1_notiming.py c2 > $o/notiming_c2.txt 2> $o/notiming_c2.err
cat $o/notiming_c1.txt $o/notiming_c2.txt
echo "r6zd done"
