#!/bin/bash
# Same-box A/B of engine builds and/or environment knobs on one config (run on the GPU box):
#     bash scripts/ab.sh OUT CFG ROUNDS VARIANT [VARIANT ...]
# VARIANT = name[:libdir][:ENV=V,ENV2=V2]   (libdir from scripts/variant.sh; '' = the default
# build).  Each round runs every variant once (interleaved, so clock drift hits all alike):
# scripts/run_config.py CFG --steps 8, printing k_scan ms, device ms per step, matched and
# selected lines.  Example:
#     bash scripts/ab.sh gpurun_out/ab c5 2 base 'nocase::KLF_QF_NO_VARIANTS=1' 'v2:klogs_amd/_lib_v2'
set -e
cd "$(dirname "$0")/.."
out=$1; cfg=$2; rounds=$3; shift 3
mkdir -p "$out"
show() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['roofline']['avg_launch_ms'], d['device_ms_per_step'], d['matched_lines'], d['selected_lines'], d['cold']['cold_ms'], d['cold']['second_run_ms'])" "$@"; }
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    IFS=: read -r name lib envs <<< "$v"
    envargs=()
    [ -n "$lib" ] && envargs+=("KLF_LIB_DIR=$lib")
    IFS=, read -ra kv <<< "$envs"
    for x in "${kv[@]}"; do [ -n "$x" ] && envargs+=("$x"); done
    env "${envargs[@]}" timeout -k 10 300 python3 scripts/run_config.py "$cfg" --steps 8 \
      > "$out/${cfg}_${name}_$r.json" 2> "$out/${cfg}_${name}_$r.err"
    show "$out/${cfg}_${name}_$r.json" "$name"
  done
done
