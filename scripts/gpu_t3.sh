# bench with the C4/C5 extras + a kernel-trace profile of the same command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-t3}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-verify > "$OUT/prof.log" 2>&1
rc=$?
echo "exit $rc" > "$OUT/rc.txt"
exit $rc
