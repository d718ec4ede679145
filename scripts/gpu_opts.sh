# A/B of libklf variants built by build_opts.sh: parity tests + scan timing per variant
# (names starting with x are timing-only ablations: no parity run).
# Usage: gpurun --timeout 900 -- bash scripts/gpu_opts.sh <tag> <name>...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for n in "$@"; do
  d=klogs_amd/_lib_o_$n; [ "$n" = base ] && d=klogs_amd/_lib
  case "$n" in x*) ;; *)
  KLF_LIB_DIR=$d timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_$n.log" 2>&1 || { echo "parity FAILED $n"; tail -30 "$OUT/pytest_$n.log"; exit 1; } ;; esac
  KLF_LIB_DIR=$d timeout -k 10 200 python3 scripts/ablate.py >> "$OUT/abl.jsonl" 2>> "$OUT/abl.err" || exit 1
done
cat "$OUT/abl.jsonl"
