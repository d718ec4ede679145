set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/t1.log 2>&1 || exit 1
(rocm-smi --showclocks 2>&1 | grep -E "sclk|mclk|fclk" >> gpurun_out/abl.jsonl || true)
timeout -k 10 120 scripts/mb_stream quick >> gpurun_out/abl.jsonl 2>&1 || exit 1
for d in klogs_amd/_lib; do
  KLF_LIB_DIR=$d timeout -k 10 300 python scripts/ablate.py >> gpurun_out/abl.jsonl 2>> gpurun_out/abl.err || exit 1
done
