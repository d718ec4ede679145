#!/bin/bash
# C5 diagnostics on the GPU box: engine counters (KLF_DIAG) and counter passes over the
# post-scan kernels.   bash scripts/diag_c5.sh OUTDIR
set -e
cd "$(dirname "$0")/.."
out=$1
export TMPDIR=/tmp
mkdir -p "$out"
KLF_DIAG=1 timeout -k 10 200 python3 scripts/run_config.py c5 --steps 1 --warmup 0 > "$out/diag.json" 2> "$out/diag.err"
bash scripts/pmc.sh "$out/pmc" c5 "k_verify|k_tindex|k_scatter|k_cmove"
