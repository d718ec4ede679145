set -e
mkdir -p gpurun_out/r5k
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pattern_counts.py tests/test_gpu_large.py -x -q --timeout 120 --timeout-method thread -k "two_level or c4 or literal or set or large" > gpurun_out/r5k/t.log 2>&1 || { tail -30 gpurun_out/r5k/t.log; exit 1; }
tail -2 gpurun_out/r5k/t.log
bash scripts/ab.sh gpurun_out/r5k c4 2 base 'noswz:klogs_amd/_lib_noswz' > gpurun_out/r5k/c4.txt 2>&1
cat gpurun_out/r5k/c4.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --kernel-include-regex "k_scan" --output-format csv -d gpurun_out/r5k/pmc -o p -- python3 scripts/run_config.py c4 --steps 2 --warmup 0 > gpurun_out/r5k/pmc.log 2>&1
python3 scripts/pmc_summary.py gpurun_out/r5k/pmc | tail -3
