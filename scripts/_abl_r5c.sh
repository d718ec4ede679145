set -e
bash scripts/ab.sh gpurun_out/r5c c5 1 base 'abl4:klogs_amd/_lib_abl4' 'abl8:klogs_amd/_lib_abl8' 'abl64:klogs_amd/_lib_abl64' 'abl128:klogs_amd/_lib_abl128' > gpurun_out/r5c/c5.txt 2>&1
bash scripts/ab.sh gpurun_out/r5c c3 1 base 'abl64:klogs_amd/_lib_abl64' > gpurun_out/r5c/c3.txt 2>&1
