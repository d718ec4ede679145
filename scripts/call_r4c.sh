set -e
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_pattern_counts.py tests/test_gpu_shard.py tests/test_gpu_compaction.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 240 python3 scripts/mall_probe.py > $O/mall.json 2> $O/mall.err; cat $O/mall.json
bash scripts/ab.sh $O/ab c3 1 base g64::KLF_GROUP_MB=64 g128::KLF_GROUP_MB=128 g256::KLF_GROUP_MB=256
bash scripts/ab.sh $O/ab c4 2 two one::KLF_QF_TWO=0
for c in c5 c4; do
KLF_DIAG=1 timeout -k 10 300 python3 scripts/run_config.py $c --steps 3 > $O/$c.json 2> $O/$c.err
grep -E "klf\] (open|run marks|first-batch|hits=)" $O/$c.err | tail -9
python3 -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['cold'], d['device_ms_per_step'], d['roofline']['avg_launch_ms'], d['stage_ms'])"
done
