# Timing-only variants of the general scan (wrong output by design) for scripts/ablate_gen.py:
#   _lib_abl4 no q-gram probes, _lib_abl8 probes without verification.
set -e
cd "$(dirname "$0")/.."
for v in 4 8; do
  d=klogs_amd/_lib_abl$v; mkdir -p $d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DKLF_ABL=$v -c klogs_amd/csrc/klf_kernels.hip -o $d/k.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $d/k.o klogs_amd/_lib/klf_engine_cpp.o klogs_amd/_lib/klf_patterns_cpp.o -o $d/libklf.so
done
