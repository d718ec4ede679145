set -e
mkdir -p gpurun_out/r5p
for c in c5 c4; do
bash scripts/ab.sh gpurun_out/r5p $c 2 base 'prio3:klogs_amd/_lib_prio3' 'prio1:klogs_amd/_lib_prio1' > gpurun_out/r5p/$c.txt 2>&1
echo "== $c"; cat gpurun_out/r5p/$c.txt
done
