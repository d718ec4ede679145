#!/bin/bash
# rocprofv3 counter passes (one pass per counter group, each its own run and time limit;
# FETCH_SIZE / WRITE_SIZE in separate passes per /opt/skills/guides/MI355X_MICROARCH.md)
# over `scripts/run_config.py CONFIG`, kernels matching REGEX:
#     scripts/pmc.sh OUTDIR CONFIG REGEX
# -> OUTDIR/<pass>/p_counter_collection.csv ; summarise with scripts/pmc_summary.py OUTDIR
set -e
cd "$(dirname "$0")/.."
out=$1; cfg=$2; rx=$3
export TMPDIR=/tmp
mkdir -p "$out"
pass() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$rx" --output-format csv -d "$out/$name" -o p \
    -- python3 scripts/run_config.py "$cfg" --steps 2 --warmup 0 > "$out/$name.log" 2>&1
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
pass sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH
pass sq3 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA
echo "pmc passes done: $out"
