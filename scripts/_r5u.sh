set -e
mkdir -p gpurun_out/r5u
for c in c5 c4; do
bash scripts/ab.sh gpurun_out/r5u $c 2 base 'abl1:klogs_amd/_lib_abl1' 'abl128:klogs_amd/_lib_abl128' > gpurun_out/r5u/$c.txt 2>&1
echo "== $c"; cat gpurun_out/r5u/$c.txt
done
