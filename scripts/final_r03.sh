#!/bin/bash
# Round-3 closing evidence on one GPU box: smoke(), the profile round's kernel traces
# (bench under rocprofv3 + C3/C4/C5 configs), and the N = 2 rehearsal of the multi-rank
# bench (gloo, both ranks on cuda:0).
set -e
cd "$(dirname "$0")/.."
out=$1
mkdir -p "$out"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
tail -2 $out/smoke.log
bash scripts/profile_round.sh "$out" trace
KLF_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > $out/bench_n2_gloo.json 2> $out/bench_n2_gloo.err
echo "final done: $out"
