set -e
mkdir -p gpurun_out/r5g
timeout -k 10 400 python -u -m pytest tests/test_gpu_timing.py tests/test_gpu_tindex.py tests/test_gpu_write.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5g/rest.log 2>&1 || { tail -30 gpurun_out/r5g/rest.log; exit 1; }
tail -2 gpurun_out/r5g/rest.log
timeout -k 10 600 python bench.py --extra-configs c3 > gpurun_out/r5g/bench.json 2> gpurun_out/r5g/bench.err
python -c "import json; d=json.load(open('gpurun_out/r5g/bench.json')); c=d['extra']['configs']['c3']; print(d['value'], d['roofline']['frac']); print({k:c.get(k) for k in ('value_GBps','ms_per_step','compaction','step_alg_frac_of_peak','verified_vs_oracle','write_path','cold','full_index')}); print(c['roofline'])"
