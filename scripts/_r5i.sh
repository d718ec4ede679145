set -e
mkdir -p gpurun_out/r5i
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pattern_counts.py tests/test_gpu_large.py -x -q --timeout 120 --timeout-method thread -k "two_level or c4 or literal or set or large" > gpurun_out/r5i/t.log 2>&1 || { tail -30 gpurun_out/r5i/t.log; exit 1; }
tail -2 gpurun_out/r5i/t.log
bash scripts/ab.sh gpurun_out/r5i c4 2 base 'old:klogs_amd/_lib_old' > gpurun_out/r5i/c4.txt 2>&1
cat gpurun_out/r5i/c4.txt
