set -e
mkdir -p gpurun_out/r5e
for c in c2 c4 c3; do
bash scripts/ab.sh gpurun_out/r5e $c 2 base 'nont:klogs_amd/_lib_nont' > gpurun_out/r5e/$c.txt 2>&1
done
