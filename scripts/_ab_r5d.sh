set -e
mkdir -p gpurun_out/r5d
bash scripts/ab.sh gpurun_out/r5d c5 2 base 'nt:klogs_amd/_lib_nt' 'sk:klogs_amd/_lib_sk' > gpurun_out/r5d/c5.txt 2>&1
