set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o kt -- python3 scripts/ablate.py > gpurun_out/kt.log 2>&1 || exit 1
