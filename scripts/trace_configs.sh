#!/bin/bash
# Kernel traces of scripts/run_config.py for the given configs (each its own time limit):
#     bash scripts/trace_configs.sh OUTDIR c2 c5 ...
set -e
cd "$(dirname "$0")/.."
out=$1; shift
export TMPDIR=/tmp
mkdir -p "$out"
for c in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace_$c" -o run \
    -- python3 scripts/run_config.py "$c" --steps 5 > "$out/run_$c.json" 2> "$out/run_$c.err"
  echo "trace $c done"
done
