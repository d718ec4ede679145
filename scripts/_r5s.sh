set -e
mkdir -p gpurun_out/r5s
for c in c4 c5; do
bash scripts/ab.sh gpurun_out/r5s $c 1 base 'abl4:klogs_amd/_lib_abl4' 'abl16:klogs_amd/_lib_abl16' 'abl64:klogs_amd/_lib_abl64' 'abl128:klogs_amd/_lib_abl128' > gpurun_out/r5s/$c.txt 2>&1
echo "== $c"; cat gpurun_out/r5s/$c.txt
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k date_edges -x -q --timeout 120 --timeout-method thread > gpurun_out/r5s/pytest.log 2>&1
tail -1 gpurun_out/r5s/pytest.log
