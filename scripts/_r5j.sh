set -e
mkdir -p gpurun_out/r5j
KLF_DIAG=1 timeout -k 10 200 python scripts/run_config.py c4 --steps 2 --warmup 0 > gpurun_out/r5j/new.json 2> gpurun_out/r5j/new.err
KLF_LIB_DIR=klogs_amd/_lib_old KLF_DIAG=1 timeout -k 10 200 python scripts/run_config.py c4 --steps 2 --warmup 0 > gpurun_out/r5j/old.json 2> gpurun_out/r5j/old.err
grep -h "blocks per CU\|hits=" gpurun_out/r5j/new.err | head -5
grep -h "blocks per CU\|hits=" gpurun_out/r5j/old.err | head -5
