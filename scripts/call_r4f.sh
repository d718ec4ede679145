set -e
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 scripts/qf_check.py --mb 32 > $O/qf.txt 2>&1; cat $O/qf.txt
bash scripts/ab.sh $O/ab c4 2 markov sketch::KLF_QF_EST=sketch
bash scripts/ab.sh $O/ab c5 1 markov sketch::KLF_QF_EST=sketch
for c in c5 c4; do
KLF_DIAG=1 timeout -k 10 300 python3 scripts/run_config.py $c --steps 3 > $O/$c.json 2> $O/$c.err
grep -E "klf\] (open: total|run marks|first-batch|hits=)" $O/$c.err | tail -6
python3 -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['cold'], d['device_ms_per_step'], d['roofline']['avg_launch_ms'], d['stage_ms'])"
done
