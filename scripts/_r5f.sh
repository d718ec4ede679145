set -e
mkdir -p gpurun_out/r5f
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5f/fused.log 2>&1 || { tail -30 gpurun_out/r5f/fused.log; exit 1; }
tail -3 gpurun_out/r5f/fused.log
timeout -k 10 200 python scripts/run_config.py c3 --steps 8 > gpurun_out/r5f/c3.json 2> gpurun_out/r5f/c3.err
python -c "import json; d=json.load(open('gpurun_out/r5f/c3.json')); print(d['compaction'], d['ms_per_step'], d['device_ms_per_step'], d['roofline'], d['step_alg_frac_of_peak'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5f/gpu_all.log 2>&1 || { tail -30 gpurun_out/r5f/gpu_all.log; exit 1; }
tail -2 gpurun_out/r5f/gpu_all.log
