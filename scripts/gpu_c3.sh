# C3 (bulk output) bench leg per libklf variant: python bench.py --extra-configs c3.
# Usage: gpurun -- bash scripts/gpu_c3.sh <tag> <name>...   (base = klogs_amd/_lib)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for n in "$@"; do
  d=klogs_amd/_lib_o_$n; [ "$n" = base ] && d=klogs_amd/_lib
  KLF_LIB_DIR=$d timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-capture --extra-configs c3 > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['extra']['configs']['c3']; print(sys.argv[2], d['value'], d['extra']['stage_ms'][3], c['value_GBps'], c['stage_ms'][3], c.get('verified_vs_c_oracle'))" "$OUT/$n.json" "$n"
done
