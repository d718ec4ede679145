#!/bin/bash
# Round-end evidence on one GPU box (each step its own time limit, chained):
#   the -m gpu suite, smoke(), the profile round (bench under rocprofv3 + config traces),
#   and an N = 2 rehearsal of the multi-rank bench (gloo, both ranks on cuda:0).
#     bash scripts/final_round.sh OUT
set -e
cd "$(dirname "$0")/.."
out=$1
mkdir -p "$out"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -1 $out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
bash scripts/profile_round.sh "$out" trace
KLF_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > $out/bench_n2_gloo.json 2> $out/bench_n2_gloo.err
echo "final_round done: $out"
