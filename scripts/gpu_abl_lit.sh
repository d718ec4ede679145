set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/abl_lit; mkdir -p $OUT
export TMPDIR=/tmp
for v in default 1 2 3; do
  if [ $v = default ]; then unset KLF_LIB_DIR; else export KLF_LIB_DIR=$PWD/klogs_amd/_lib_abl$v; fi
  timeout -k 10 200 python -u scripts/ablate.py >> $OUT/res.jsonl 2>> $OUT/err.log || exit $?
done
