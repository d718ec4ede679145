# A/B of the k_cgather unroll (KLF_COPY_U) on C3: parity subset + bench per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for n in "$@"; do
  d=klogs_amd/_lib_o_$n; [ "$n" = base ] && d=klogs_amd/_lib
  KLF_LIB_DIR=$d timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_write.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_$n.log" 2>&1 || { echo "parity FAILED $n"; tail -30 "$OUT/pytest_$n.log"; exit 1; }
  KLF_LIB_DIR=$d timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-capture --extra-configs c3 > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || exit 1
done
