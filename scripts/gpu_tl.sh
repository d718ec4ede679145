cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python scripts/timeline.py > gpurun_out/tl.log 2>&1
