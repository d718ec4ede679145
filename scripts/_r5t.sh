set -e
mkdir -p gpurun_out/r5t
bash scripts/ab.sh gpurun_out/r5t c4 2 new 'old:klogs_amd/_lib_old' > gpurun_out/r5t/c4.txt 2>&1
echo "== c4"; cat gpurun_out/r5t/c4.txt
