# parity suite + C2 bench (no extras) + general-set timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-t6}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --extra-configs "" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
KLF_DIAG=1 timeout -k 10 200 python -u scripts/ablate_gen.py > $OUT/abl.json 2> $OUT/err.log
