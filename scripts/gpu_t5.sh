set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-t5}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit $?
KLF_DIAG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 scripts/ablate_gen.py > "$OUT/abl.json" 2> "$OUT/err.log"
