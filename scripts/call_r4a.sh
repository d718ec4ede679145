set -e
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
for c in c5 c4; do
KLF_DIAG=1 timeout -k 10 300 python3 scripts/run_config.py $c --steps 3 > $O/$c.json 2> $O/$c.err
grep -E "klf\] (open|run)" $O/$c.err | tail -12
python3 -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['cold'], d['device_ms_per_step'], d['roofline']['avg_launch_ms'])"
done
