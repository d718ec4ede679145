set -e
mkdir -p gpurun_out/r5n
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5n/gpu_all.log 2>&1 || { tail -30 gpurun_out/r5n/gpu_all.log; exit 1; }
tail -2 gpurun_out/r5n/gpu_all.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5n/smoke.log 2>&1
tail -1 gpurun_out/r5n/smoke.log
