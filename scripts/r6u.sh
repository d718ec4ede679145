#!/bin/bash
# Round 6: k_verify at 4 waves per SIMD (<= 128 VGPRs), entries 4 / 2 at once (C4, C5 same box)
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6u; mkdir -p $o
bash scripts/ktrace_ab.sh $o c4 base w4:klogs_amd/_lib_vw4 w4e2:klogs_amd/_lib_vw4e2 base2 > $o/kt_c4.txt 2>&1
bash scripts/ktrace_ab.sh $o c5 base w4:klogs_amd/_lib_vw4 w4e2:klogs_amd/_lib_vw4e2 > $o/kt_c5.txt 2>&1
echo "r6u done"
