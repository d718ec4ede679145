# SQ counter passes over bench.py (one pass per run) + the streaming calibration.
# Usage: gpurun -- bash scripts/gpu_pmc_bench.sh <tag> [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-pmc}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify $*"
hipcc --offload-arch=gfx950 -O3 scripts/mb_stream.hip -o /tmp/mb_stream &&
timeout -k 10 120 /tmp/mb_stream quick > "$OUT/mb_stream.txt" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d "$OUT/p1" -o p --output-format csv -- $B > "$OUT/p1.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH -d "$OUT/p2" -o p --output-format csv -- $B > "$OUT/p2.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC -d "$OUT/p3" -o p --output-format csv -- $B > "$OUT/p3.log" 2>&1
rc=$?
echo "exit $rc" > "$OUT/rc.txt"
exit $rc
