# Timing-only variants of the general scan (wrong output by design) for scripts/ablate_gen.py:
#   _lib_abl16 k_verify without verification work, _lib_abl32 bucket walks only.
set -e
cd "$(dirname "$0")/.."
for v in 16 32; do
  d=klogs_amd/_lib_abl$v; mkdir -p $d
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DKLF_ABL=$v -c klogs_amd/csrc/klf_kernels.hip -o $d/k.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $d/k.o klogs_amd/_lib/klf_engine_cpp.o klogs_amd/_lib/klf_patterns_cpp.o -o $d/libklf.so
done
