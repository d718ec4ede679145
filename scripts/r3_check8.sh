#!/bin/bash
# k_cmove grid size: kernel traces of C2 and C5 with KLF_CG_GRID 8 (default), 2, 1
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "short_lines or clamped or dense_tiles" -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
tail -1 $out/pytest.log
for L in _lib _lib_cg2 _lib_cg1; do for c in c2 c5; do
  KLF_LIB_DIR=klogs_amd/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/tr_${c}$L -o run -- python3 scripts/run_config.py $c --steps 5 > $out/${c}$L.json 2> $out/${c}$L.err
  python3 -c "import csv,sys; r=[x for x in csv.DictReader(open(sys.argv[1])) if 'k_cmove' in x['Name'] or 'k_cplan' in x['Name'] or 'k_cmid' in x['Name']]; print(sys.argv[2], [(x['Name'][:30], round(float(x['AverageNs'])/1e3,1)) for x in r])" $out/tr_${c}$L/run_kernel_stats.csv $c$L
done; done
