# GPU parity (full -m gpu suite) + a short bench; used while iterating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-t2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest exit $rc" > "$OUT/rc.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
echo "bench exit $rc" >> "$OUT/rc.txt"
exit $rc
