set -e
O=gpurun_out/r4b; mkdir -p $O
timeout -k 10 60 ./scripts/mb_depth > $O/mb_depth.txt 2>&1; cat $O/mb_depth.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pattern_counts.py tests/test_gpu_staging.py tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for c in c5 c4; do
KLF_DIAG=1 timeout -k 10 300 python3 scripts/run_config.py $c --steps 3 > $O/$c.json 2> $O/$c.err
grep -E "klf\] (open|run marks|first-batch)" $O/$c.err | tail -8
python3 -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['cold'], d['device_ms_per_step'], d['roofline']['avg_launch_ms'])"
done
bash scripts/ab.sh $O/ab c4 1 base a4:klogs_amd/_lib_a4 a8:klogs_amd/_lib_a8 a64:klogs_amd/_lib_a64
bash scripts/ab.sh $O/ab c5 1 base a4:klogs_amd/_lib_a4 a8:klogs_amd/_lib_a8 a64:klogs_amd/_lib_a64
