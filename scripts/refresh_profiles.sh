# Copies one gpu_round.sh result (gpurun_out/<tag>) into profiles/r01 and recomputes the
# per-launch HBM traffic of the dominant kernel from its FETCH_SIZE / WRITE_SIZE passes.
# Usage: bash scripts/refresh_profiles.sh <tag>
set -e
cd "$(dirname "$0")/.."
IN=gpurun_out/$1
P=profiles/r01
cp "$IN/bench.json" $P/bench.json
cp "$IN/prof/run_kernel_stats.csv" $P/bench_kernel_stats.csv
cp "$IN/pmc_fetch/p_counter_collection.csv" $P/pmc_fetch_size.csv
cp "$IN/pmc_write/p_counter_collection.csv" $P/pmc_write_size.csv
cp "$IN/pytest_gpu.log" $P/pytest_gpu.log
cp "$IN/smoke.log" $P/smoke.log
python3 scripts/pmc_traffic.py $P/pmc_fetch_size.csv $P/pmc_write_size.csv $P/traffic.json
