# §8f-3 write path: its GPU tests, the CLI tests that now write through it, and the C3 bench leg.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-w1}
mkdir -p "$OUT"
export TMPDIR=/tmp
df -h /tmp /dev/shm > "$OUT/df.txt" 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_write.py tests/test_gpu_host.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-capture --extra-configs c3 > "$OUT/bench.json" 2> "$OUT/bench.err"
