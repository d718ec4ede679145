#!/bin/bash
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
bash scripts/ab_lib.sh $out c3 klogs_amd/_lib_prev klogs_amd/_lib_tc4 2
bash scripts/ab_lib.sh $out c3 klogs_amd/_lib_tc2 klogs_amd/_lib 1
