set -e
mkdir -p gpurun_out/r5m
KLF_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r5m/bench_n2_gloo.json 2> gpurun_out/r5m/bench_n2_gloo.err
python -c "
import json; d=json.load(open('gpurun_out/r5m/bench_n2_gloo.json'))
print(d['value'], d['n_gpus'], d['ms_per_step'], d['roofline']['frac'], d['config']['workload'][:60])
h=d['extra']['headline']; print({k:h[k] for k in ('records_consistent','verified_vs_oracle','step_alg_frac_of_peak_per_gpu','scan_frac_min_over_ranks')})
for k,v in d['extra']['configs'].items(): print(k, v['value_GBps'], v['ms_per_step'], v.get('records_consistent'), v.get('verified_vs_oracle'))
"
