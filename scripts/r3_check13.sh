#!/bin/bash
# k_scatter grid: kernel traces of C5, C3, C2 with KLF_SCATTER_GRID 8 (default), 16, 32
set -e
cd "$(dirname "$0")/.."
out=$1; mkdir -p $out
export TMPDIR=/tmp
for c in c5 c3 c2; do for L in _lib _lib_sg16 _lib_sg32; do
  KLF_LIB_DIR=klogs_amd/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/tr_${c}$L -o run -- python3 scripts/run_config.py $c --steps 4 > $out/${c}$L.json 2> /dev/null
  python3 -c "import csv,sys,json; r=[x for x in csv.DictReader(open(sys.argv[1])) if 'k_scatter' in x['Name']]; d=json.load(open(sys.argv[3])); print(sys.argv[2], [round(float(x['AverageNs'])/1e3,1) for x in r], d['device_ms_per_step'])" $out/tr_${c}$L/run_kernel_stats.csv $c$L $out/${c}$L.json
done; done
