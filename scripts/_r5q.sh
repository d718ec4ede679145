set -e
mkdir -p gpurun_out/r5q
bash scripts/ab.sh gpurun_out/r5q c5 2 base 'two::KLF_QF_TWO=force' > gpurun_out/r5q/c5.txt 2>&1
cat gpurun_out/r5q/c5.txt
KLF_DIAG=1 KLF_QF_TWO=force timeout -k 10 200 python3 scripts/run_config.py c5 --steps 2 > gpurun_out/r5q/diag.json 2> gpurun_out/r5q/diag.err
grep -i 'layout\|hits' gpurun_out/r5q/diag.err | head -20
