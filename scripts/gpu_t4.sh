set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-t4}; mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit $?
for v in default; do
  if [ $v = default ]; then unset KLF_LIB_DIR; else export KLF_LIB_DIR=$PWD/klogs_amd/_lib_abl$v; fi
  KLF_DIAG=1 timeout -k 10 200 python -u scripts/ablate_gen.py >> $OUT/abl.jsonl 2>> $OUT/err.log || exit $?
done
