#!/bin/bash
# Builds a timing/diagnostic variant of libklf.so: scripts/variant.sh NAME -DKNOB=V ...
# -> klogs_amd/_lib_NAME/libklf.so (select it with KLF_LIB_DIR=klogs_amd/_lib_NAME).
# Variants with ablation knobs compute wrong output by design; they only time kernels.
set -e
cd "$(dirname "$0")/.."
name=$1; shift
python3 -c "from klogs_amd import _build; _build.build_engine()"
d=klogs_amd/_lib_$name; mkdir -p $d
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c klogs_amd/csrc/klf_kernels.hip -o $d/k.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $d/k.o klogs_amd/_lib/klf_engine_cpp.o klogs_amd/_lib/klf_patterns_cpp.o -o $d/libklf.so
rm -f $d/k.o
