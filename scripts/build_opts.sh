# Builds libklf variants for A/B timing: each arg is NAME=FLAGS, e.g. o1="-DKLF_OPT=1".
# Output: klogs_amd/_lib_o_NAME/libklf.so (git-ignored; travels with gpurun).
set -e
cd "$(dirname "$0")/.."
python3 -c "import __graft_entry__ as g; g.build()"
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  d=klogs_amd/_lib_o_$name; mkdir -p $d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function $flags -c klogs_amd/csrc/klf_kernels.hip -o $d/k.o &
done
wait
for spec in "$@"; do
  name=${spec%%=*}; d=klogs_amd/_lib_o_$name
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $d/k.o klogs_amd/_lib/klf_engine_cpp.o klogs_amd/_lib/klf_patterns_cpp.o -o $d/libklf.so
  rm -f $d/k.o
done
