#!/bin/bash
# Per-kernel times of build / environment variants on one config, same box (run on the GPU
# box): a rocprofv3 kernel trace of scripts/run_config.py CFG per variant, then the split.
#     bash scripts/ktrace_ab.sh OUT CFG VARIANT [VARIANT ...]
# VARIANT = name[:libdir][:ENV=V,ENV2=V2]  (as scripts/ab.sh; libdir from scripts/variant.sh)
set -e
cd "$(dirname "$0")/.."
out=$1; cfg=$2; shift 2
export TMPDIR=/tmp
mkdir -p "$out"
for v in "$@"; do
  IFS=: read -r name lib envs <<< "$v"
  envargs=()
  [ -n "$lib" ] && envargs+=("KLF_LIB_DIR=$lib")
  IFS=, read -ra kv <<< "$envs"
  for x in "${kv[@]}"; do [ -n "$x" ] && envargs+=("$x"); done
  env "${envargs[@]}" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/t_${cfg}_$name" -o run \
    -- python3 scripts/run_config.py "$cfg" --steps 6 > "$out/${cfg}_$name.json" 2> "$out/${cfg}_$name.err"
  echo "== $cfg $name"
  python3 scripts/kernel_split.py "$(ls "$out"/t_${cfg}_$name/*/run_kernel_trace.csv "$out"/t_${cfg}_$name/run_kernel_trace.csv 2>/dev/null | head -1)" | head -14
done
