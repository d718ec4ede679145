set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/abl_gen; mkdir -p $OUT
export TMPDIR=/tmp
for v in default 4 8; do
  if [ $v = default ]; then unset KLF_LIB_DIR; else export KLF_LIB_DIR=$PWD/klogs_amd/_lib_abl$v; fi
  timeout -k 10 200 python -u scripts/ablate_gen.py >> $OUT/res.jsonl 2>> $OUT/err.log || exit $?
done
