set -e
mkdir -p gpurun_out/r5o
for c in c5 c2 c4; do
KLF_DIAG=1 timeout -k 10 200 python scripts/cold_diag.py $c > gpurun_out/r5o/$c.txt 2> gpurun_out/r5o/$c.err
echo "== $c"; cat gpurun_out/r5o/$c.txt
done
