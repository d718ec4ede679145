set -e
mkdir -p gpurun_out/r5h
bash scripts/ab.sh gpurun_out/r5h c4 1 base 'abl4:klogs_amd/_lib_abl4' 'abl16:klogs_amd/_lib_abl16' 'abl64:klogs_amd/_lib_abl64' > gpurun_out/r5h/c4.txt 2>&1
KLF_DIAG=1 timeout -k 10 200 python scripts/run_config.py c5 --steps 3 --warmup 0 > gpurun_out/r5h/c5diag.json 2> gpurun_out/r5h/c5diag.err
KLF_DIAG=1 timeout -k 10 200 python scripts/run_config.py c3 --steps 3 --warmup 0 > gpurun_out/r5h/c3diag.json 2> gpurun_out/r5h/c3diag.err
KLF_DIAG=1 timeout -k 10 200 python scripts/run_config.py c2 --steps 3 --warmup 0 > gpurun_out/r5h/c2diag.json 2> gpurun_out/r5h/c2diag.err
cat gpurun_out/r5h/c4.txt
