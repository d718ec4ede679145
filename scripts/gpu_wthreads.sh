# Writer-thread count of klf_result_write on the C3 output (8 vs 16 vs 4).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-wt}
mkdir -p "$OUT"
export TMPDIR=/tmp
for n in 8 16 4; do
  KLF_WRITE_THREADS=$n timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-capture --extra-configs c3 > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || exit 1
done
