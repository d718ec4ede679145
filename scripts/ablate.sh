#!/bin/bash
# Times timing-variant builds (scripts/variant.sh) on BASELINE configs, on the GPU box:
#     bash scripts/ablate.sh OUT "base noslot ..." "c2 c5 ..."
# -> OUT/<variant>_<cfg>.json (scripts/run_config.py lines; roofline.avg_launch_ms = k_scan)
set -e
cd "$(dirname "$0")/.."
out=$1; vars=$2; cfgs=$3
mkdir -p "$out"
for c in $cfgs; do
  for v in $vars; do
    KLF_LIB_DIR=klogs_amd/_lib_$v timeout -k 10 240 python3 scripts/run_config.py "$c" --steps 5 --warmup 2 \
      > "$out/${v}_$c.json" 2> "$out/${v}_$c.err"
    echo "$v $c $(python3 -c "import json,sys; d=json.load(open('$out/${v}_$c.json')); print(d['roofline']['avg_launch_ms'], d['device_ms_per_step'])")"
  done
done
