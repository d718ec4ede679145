#!/bin/bash
# One round's profiles, on the GPU box (each step its own time limit, chained):
#     bash scripts/profile_round.sh OUT [trace|pmc|all]
#   OUT/trace   rocprofv3 --kernel-trace --stats of the driver's exact bench command
#   OUT/bench.json, bench.err   that run's bench line
#   OUT/trace_<cfg>             kernel traces of scripts/run_config.py for C3 and C5
#   OUT/pmc_<cfg>/...           counter passes (scripts/pmc.sh) for C2, C3 and C5
# then, in the build container: python3 scripts/collect_profiles.py OUT profiles/rNN
set -e
cd "$(dirname "$0")/.."
out=$1
what=${2:-all}
export TMPDIR=/tmp
mkdir -p "$out"
if [ "$what" != pmc ]; then
  timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run \
    -- python3 bench.py > "$out/bench.json" 2> "$out/bench.err"
  echo "trace done"
  for c in c5 c2 c3 c4; do  # per-config kernel splits (the bench trace mixes every config)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace_$c" -o run \
      -- python3 scripts/run_config.py "$c" --steps 8 > "$out/run_$c.json" 2> "$out/run_$c.err"
    echo "trace $c done"
  done
fi
if [ "$what" != trace ]; then
  for c in c2 c3 c4 c5; do
    bash scripts/pmc.sh "$out/pmc_$c" "$c" "k_scan|k_tcopy|k_cplan|k_cmove|k_tindex|k_scatter|k_verify|k_nfa"
  done
fi
echo "profile_round done: $out"
