# Compaction change check: full GPU parity suite, then the bench (C2 + C3 extra).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-cmp}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-capture --extra-configs c3,c4,c5 > "$OUT/bench.json" 2> "$OUT/bench.err"
