#!/bin/bash
# k_cmove with and without its copy loop (timing build), C5 and C2 kernel traces.
set -e
cd "$(dirname "$0")/.."
out=$1
mkdir -p $out
export TMPDIR=/tmp
for v in base nocopy; do
  d=klogs_amd/_lib; [ $v = nocopy ] && d=klogs_amd/_lib_nocopy
  KLF_LIB_DIR=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$v" -o run \
    -- python3 scripts/run_config.py c5 --steps 5 > "$out/$v.json" 2> "$out/$v.err"
  echo "$v done"
done
