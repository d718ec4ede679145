#!/bin/bash
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pattern_counts.py tests/test_gpu_large.py tests/test_gpu_tindex.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
tail -1 $out/pytest.log
bash scripts/ab_lib.sh $out c5 klogs_amd/_lib_prev klogs_amd/_lib 2
for L in _lib_prev _lib; do
  KLF_LIB_DIR=klogs_amd/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/tr_c5$L -o run -- python3 scripts/run_config.py c5 --steps 4 > /dev/null 2>&1
  python3 -c "import csv,sys; r=[x for x in csv.DictReader(open(sys.argv[1])) if 'k_verify' in x['Name'] or 'k_nfa' in x['Name']]; print(sys.argv[2], [(x['Name'][27:40], round(float(x['AverageNs'])/1e3,1)) for x in r])" $out/tr_c5$L/run_kernel_stats.csv $L
done
