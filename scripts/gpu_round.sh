# One GPU call: parity tests, smoke, bench (C2 headline + C4/C5 extras), kernel-trace
# profile of the C2 bench, HBM counter passes (FETCH_SIZE / WRITE_SIZE, separate runs).
# Usage (from the CPU container): gpurun --timeout 1200 -- bash scripts/gpu_round.sh [tag]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "host cpus: $(nproc)" > "$OUT/host.txt"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 500 python -u bench.py --steps 20 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-verify --no-capture --extra-configs "" > "$OUT/prof.log" 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-capture --extra-configs "" > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o p --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-capture --extra-configs "" > "$OUT/pmc_write.log" 2>&1
rc=$?
echo "exit $rc" > "$OUT/rc.txt"
exit $rc
