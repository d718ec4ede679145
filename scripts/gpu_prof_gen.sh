set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-prof_gen}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 scripts/ablate_gen.py > "$OUT/abl.json" 2> "$OUT/err.log"
