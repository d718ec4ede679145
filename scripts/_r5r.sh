set -e
mkdir -p gpurun_out/r5r
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5r/pytest_gpu.log 2>&1
tail -1 gpurun_out/r5r/pytest_gpu.log
for c in c5 c2 c3; do
bash scripts/ab.sh gpurun_out/r5r $c 2 new 'old:klogs_amd/_lib_old' > gpurun_out/r5r/$c.txt 2>&1
echo "== $c"; cat gpurun_out/r5r/$c.txt
done
