# Scan ablations (timing + VALU/SALU counts) and post-scan stage diagnostics.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-abl}
mkdir -p "$OUT"
export TMPDIR=/tmp
for d in _lib _lib_abl1 _lib_abl2 _lib_abl3; do
  KLF_LIB_DIR=klogs_amd/$d timeout -k 10 200 python3 scripts/ablate.py >> "$OUT/abl.jsonl" 2>> "$OUT/abl.err" || exit 1
  KLF_LIB_DIR=klogs_amd/$d timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d "$OUT/pmc$d" -o p --output-format csv -- python3 scripts/ablate.py > "$OUT/pmc$d.log" 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/post" -o p --output-format csv -- python3 scripts/diag_post.py > "$OUT/post.log" 2>&1
