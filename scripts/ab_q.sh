#!/bin/bash
# same-box A/B of the prefilter gram length on C5 (4-byte vs 3-byte grams)
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
show() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['roofline']['avg_launch_ms'], d['device_ms_per_step'], d['matched_lines'], d['selected_lines'])" "$@"; }
for r in 1 2; do for q in 4 3; do
  KLF_QF_QMAX=$q timeout -k 10 240 python3 scripts/run_config.py c5 --steps 8 > $out/c5_q${q}_$r.json 2> $out/c5_q${q}_$r.err
  show $out/c5_q${q}_$r.json q$q
done; done
