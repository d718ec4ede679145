#!/bin/bash
# same-box A/B of two builds on one config: bash scripts/ab_lib.sh OUT CFG LIBDIR_A LIBDIR_B [rounds]
set -e
cd "$(dirname "$0")/.."
out=$1; cfg=$2; A=$3; B=$4; n=${5:-2}; mkdir -p $out
show() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['roofline']['avg_launch_ms'], d['device_ms_per_step'], d['matched_lines'], d['selected_lines'])" "$@"; }
for r in $(seq 1 $n); do for L in $A $B; do
  t=$(basename $L)
  KLF_LIB_DIR=$L timeout -k 10 240 python3 scripts/run_config.py $cfg --steps 8 > $out/${cfg}_${t}_$r.json 2> $out/${cfg}_${t}_$r.err
  show $out/${cfg}_${t}_$r.json $t
done; done
