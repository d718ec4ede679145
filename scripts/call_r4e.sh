set -e
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash scripts/ab.sh $O/ab c3 2 lazy full::KLF_LAZY_INDEX=0
KLF_DIAG=1 timeout -k 10 300 python3 scripts/run_config.py c5 --steps 3 > $O/c5.json 2> $O/c5.err
grep -E "klf\] open" $O/c5.err
