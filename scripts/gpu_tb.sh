set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/t1.log 2>&1
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
if [ -d klogs_amd/_lib_b ]; then KLF_LIB_DIR=klogs_amd/_lib_b timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err; fi
