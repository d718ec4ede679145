set -e
mkdir -p gpurun_out/r5v
bash scripts/ab.sh gpurun_out/r5v c4 3 defer 'nodefer:klogs_amd/_lib_nodefer' > gpurun_out/r5v/c4.txt 2>&1
echo "== c4"; cat gpurun_out/r5v/c4.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pattern_counts.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5v/pytest.log 2>&1
tail -1 gpurun_out/r5v/pytest.log
