#!/bin/bash
# plain / literal scan occupancy (launch bounds) on C2 and C3
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
bash scripts/ab_lib.sh $out c2 klogs_amd/_lib klogs_amd/_lib_occ3 2
bash scripts/ab_lib.sh $out c2 klogs_amd/_lib_occ5 klogs_amd/_lib 1
bash scripts/ab_lib.sh $out c3 klogs_amd/_lib klogs_amd/_lib_occ3 1
bash scripts/ab_lib.sh $out c3 klogs_amd/_lib_occ5 klogs_amd/_lib 1
