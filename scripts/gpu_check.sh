# Parity tests + default bench (sanity check of the in-tree build).
# Usage: gpurun --timeout 900 -- bash scripts/gpu_check.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-check}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --extra-configs "" > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-verify --extra-configs "" > "$OUT/prof.log" 2>&1
rc=$?
echo "exit $rc" > "$OUT/rc.txt"
tail -3 "$OUT/pytest_gpu.log"
exit $rc
