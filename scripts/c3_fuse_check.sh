#!/bin/bash
# C3 fused vs two-pass: the fused-compaction GPU tests, then kernel traces of C3 both ways.
#     bash scripts/c3_fuse_check.sh OUT
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_compaction.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
tail -1 $out/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/tr_fused -o run -- python3 scripts/run_config.py c3 --steps 5 > $out/c3_fused.json 2> $out/c3_fused.err
KLF_FUSE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/tr_two -o run -- python3 scripts/run_config.py c3 --steps 5 > $out/c3_two.json 2> $out/c3_two.err
echo traces done
bash scripts/ablate.sh $out/abl "a4096 a4 a128 a64" "c4" > $out/abl_c4.txt 2>&1
bash scripts/ablate.sh $out/abl "a4096 a4" "c5" > $out/abl_c5.txt 2>&1
echo ablations done
KLF_DIAG=1 timeout -k 10 240 python3 scripts/run_config.py c5 --steps 2 > $out/diag_c5.json 2> $out/diag_c5.err
KLF_DIAG=1 timeout -k 10 240 python3 scripts/run_config.py c4 --steps 2 > $out/diag_c4.json 2> $out/diag_c4.err
echo diag done
