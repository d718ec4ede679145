# Parity tests, then scan timing (ablate.py) and post-scan stage split (diag_post.py).
# Usage: gpurun --timeout 900 -- bash scripts/gpu_quick.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-quick}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 200 python3 scripts/ablate.py > "$OUT/abl.jsonl" 2> "$OUT/abl.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/post" -o p --output-format csv -- python3 scripts/diag_post.py > "$OUT/post.log" 2>&1
rc=$?
echo "exit $rc" > "$OUT/rc.txt"
tail -3 "$OUT/pytest_gpu.log"
exit $rc
