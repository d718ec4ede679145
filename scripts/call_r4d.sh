set -e
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 240 python3 scripts/mall_probe.py > $O/mall.json 2> $O/mall.err; cat $O/mall.json
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err; tail -c 400 $O/bench.json; echo
KLF_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err
python3 -c "import json; d=json.loads(open('$O/bench_n2_gloo.json').read().strip().splitlines()[-1]); print(d['value'], d['extra']['verified_vs_c_oracle'], {k:(v.get('value_GBps'), v.get('verified_vs_oracle'), v.get('records_consistent')) for k,v in d['extra']['configs'].items()})"
