# Kernel-level times (rocprofv3 kernel trace) of scripts/ablate.py for libklf variants.
# Usage: gpurun -- bash scripts/gpu_ktime.sh <tag> <name>...   (base = klogs_amd/_lib)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for n in "$@"; do
  d=klogs_amd/_lib_o_$n; [ "$n" = base ] && d=klogs_amd/_lib
  KLF_LIB_DIR=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$n" -o k --output-format csv -- python3 scripts/ablate.py > "$OUT/$n.log" 2>&1 || exit 1
  echo "== $n"; cut -d, -f1-4 "$OUT/$n"/*/k_kernel_stats.csv 2>/dev/null | head -14 || find "$OUT/$n" -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \; | head -14
done
